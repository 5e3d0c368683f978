// stream_probe.hip — isolates what limits the Net pass's staging loop (tool, not product).
// Each wave streams 64-record tiles of 80-B records (5 KiB) like the Net pass, one tile
// of register prefetch ahead, workgroup b owning a contiguous tile range.
//   mode 0: addresses from arithmetic, 5 x 16-B loads per lane
//   mode 1: + a 6th load that re-reads the tile's last chunk (clamped lanes)
//   mode 2: + tile bounds from per-lane loads of a record-offset array (two loads per
//           lane per tile, one tile further ahead, readlane for the bounds)
//   mode 3: mode 2 + LDS commit of the tile (ds_write_b128)
//   mode 4: mode 3 + an 8-B per-lane store per tile (dense IP log)
//   mode 5: mode 4 + two 16-B per-lane stores per tile into a per-wave 2-KiB area
//   mode 6: mode 4 + two 16-B stores per tile, all lanes of a wave to one address
//   mode 7: mode 2 with per-lane windows: each lane loads its own record's 80 B (five
//           16-B loads from the 16-B aligned record start), no LDS
//   mode 8: mode 7 from the dword-aligned record start (unaligned 16-B loads)
// usage: stream_probe [records]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define REC 80
#define WT 64

template <int MODE>
__global__ void __launch_bounds__(256) probe(const uint8_t *__restrict__ recs, const uint32_t *__restrict__ offs,
                                             uint64_t n, uint64_t wtpb, uint32_t *out, uint64_t *log)
{
    __shared__ uint4 stage[4][6 * 64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t nwt = (n + WT - 1) / WT;
    const uint64_t wbeg = blockIdx.x * wtpb, wend = min(wbeg + wtpb, nwt);
    const uint64_t last = n - 1;
    uint32_t acc = 0;
    constexpr int NJ = (MODE == 0 || MODE >= 7) ? 5 : 6;
    uint4 pf[NJ];
#define ISSUE(B0, B1)                                                                  \
    {                                                                                  \
        const uint32_t b0_ = (B0), nch_ = ((B1) - b0_ + 15) >> 4;                       \
        _Pragma("unroll") for (int j = 0; j < NJ; j++)                                 \
        {                                                                              \
            const uint32_t ch = min((uint32_t)(j * 64) + lane, nch_ - 1);              \
            pf[j] = *reinterpret_cast<const uint4 *>(recs + b0_ + ch * 16);            \
        }                                                                              \
    }
    auto lane_off = [&](uint64_t t) -> uint32_t { return offs[min(t * WT + lane, last)]; };
    auto lane_end = [&](uint64_t t) -> uint32_t { return offs[min(t * WT + lane + 1, last)]; };
    uint64_t t = wbeg + wave;
    uint32_t off_n = 0, end_n = 0;
    if (t < wend) {
        if (MODE >= 7) {
            const uint32_t o0 = lane_off(t);
            const uint32_t a = MODE == 7 ? (o0 & ~15u) : (o0 & ~3u);
#pragma unroll
            for (int j = 0; j < NJ; j++) pf[j] = *reinterpret_cast<const uint4 *>(recs + a + 16 * j);
            off_n = lane_off(t + 4);
        } else if (MODE >= 2) {
            const uint32_t o0 = lane_off(t), e0 = lane_end(t);
            ISSUE(__builtin_amdgcn_readlane(o0, 0), __builtin_amdgcn_readlane(e0, 63));
            off_n = lane_off(t + 4);
            end_n = lane_end(t + 4);
        } else {
            ISSUE((uint32_t)(t * WT * REC), (uint32_t)((t + 1) * WT * REC));
        }
    }
    for (; t < wend; t += 4) {
        if (MODE >= 3 && MODE < 7) {
#pragma unroll
            for (int j = 0; j < NJ; j++) stage[wave][j * 64 + lane] = pf[j];
        } else {
#pragma unroll
            for (int j = 0; j < NJ; j++) acc += pf[j].x ^ pf[j].y ^ pf[j].z ^ pf[j].w;
        }
        if (t + 4 < wend) {
            if (MODE >= 7) {
                const uint32_t a = MODE == 7 ? (off_n & ~15u) : (off_n & ~3u);
#pragma unroll
                for (int j = 0; j < NJ; j++) pf[j] = *reinterpret_cast<const uint4 *>(recs + a + 16 * j);
                off_n = lane_off(t + 8);
            } else if (MODE >= 2) {
                ISSUE(__builtin_amdgcn_readlane(off_n, 0), __builtin_amdgcn_readlane(end_n, 63));
                off_n = lane_off(t + 8);
                end_n = lane_end(t + 8);
            } else {
                ISSUE((uint32_t)((t + 4) * WT * REC), (uint32_t)((t + 5) * WT * REC));
            }
        }
        if (MODE >= 3 && MODE < 7) acc += stage[wave][(lane * 5) % 320].x;
        if (MODE >= 4 && MODE < 7) log[t * WT + lane] = acc;
        if (MODE == 5) { uint4 *tr = reinterpret_cast<uint4 *>(log + 20000000) + (blockIdx.x * 4 + wave) * 128; tr[lane] = pf[0]; tr[64 + lane] = pf[1]; }
        if (MODE == 6) { uint4 *tr = reinterpret_cast<uint4 *>(log + 20000000) + (blockIdx.x * 4 + wave) * 2; tr[0] = pf[0]; tr[1] = pf[1]; }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
    const size_t bytes = n * REC + 256;
    uint8_t *d;
    uint32_t *o, *offs;
    uint64_t *log;
    hipMalloc(&d, bytes);
    hipMalloc(&o, 4);
    hipMalloc(&offs, n * 4);
    hipMalloc(&log, (n + 64) * 8 + (64ull << 20));
    hipMemset(d, 1, bytes);
    std::vector<uint32_t> h(n);
    for (uint64_t i = 0; i < n; i++) h[i] = (uint32_t)(i * REC);
    hipMemcpy(offs, h.data(), n * 4, hipMemcpyHostToDevice);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint64_t nwt = (n + WT - 1) / WT;
    for (int mode = 0; mode < 9; mode++)
        for (int wpc : {2, 4, 8}) {
            const uint64_t grid = (uint64_t)cus * wpc;
            const uint64_t wtpb = (nwt + grid - 1) / grid;
            float best = 1e9f;
            for (int it = 0; it < 6; it++) {
                hipEventRecord(a);
                switch (mode) {
                case 0: hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 1: hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 2: hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 3: hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 4: hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 5: hipLaunchKernelGGL(probe<5>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 6: hipLaunchKernelGGL(probe<6>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                case 7: hipLaunchKernelGGL(probe<7>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                default: hipLaunchKernelGGL(probe<8>, dim3(grid), dim3(256), 0, 0, d, offs, n, wtpb, o, log); break;
                }
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (it > 0 && ms < best) best = ms;
            }
            printf("mode %d wg/cu=%d  %.1f us  %.0f GB/s\n", mode, wpc, best * 1e3, n * (double)REC / (best * 1e-3) / 1e9);
        }
    return 0;
}
