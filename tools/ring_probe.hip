// ring_probe.hip — how many bytes in flight per CU the Net pass's record staging needs
// (tool, not product). 10M 80-B records (C2 shape), 64-record tiles, each lane ends with its
// record's first 64 bytes in registers (XOR-folded so nothing is dead), optional 4-B store per
// record (the compact IP log). Workgroup b owns a contiguous tile range; wave w of NW takes
// tiles w, w + NW, ... of it.
//   plain      : coalesced 16-B loads over the blob (ceiling)
//   reg        : the product's register windows (5 x 16-B loads per lane from the record start,
//                offsets two tiles ahead, two window buffers)
//   ring<Q,NJ> : per-wave LDS ring of Q tile slots filled by LDS-DMA (global_load_lds_dwordx4,
//                NJ 1-KiB contiguous pieces per tile from the tile's 16-B aligned span start),
//                offset rows by LDS-DMA 2Q tiles ahead, exact vmcnt waits; Q - 1 tiles in flight
//                while one is parsed; records read back with five ds_read_b128
// usage: ring_probe [records]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define REC 80
#define WT 64

__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p);
}
__device__ __forceinline__ void dma16(const void *gsrc, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(const void *gsrc, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t fold(const uint4 (&W)[5], uint32_t sh)
{
    uint32_t x[17];
#pragma unroll
    for (int k = 0; k < 4; k++) { x[4 * k] = W[k].x; x[4 * k + 1] = W[k].y; x[4 * k + 2] = W[k].z; x[4 * k + 3] = W[k].w; }
    x[16] = W[4].x;
    uint32_t a = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) a = (a << 1 | a >> 31) ^ __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
    return a;
}

__global__ void __launch_bounds__(256) plain(const uint4 *__restrict__ p, uint64_t n16, uint32_t *out)
{
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n16; i += 8 * stride) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = p[i + u * stride];
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) acc ^= p[i].x;
    if (acc == 0x12345678u) out[0] = acc;
}

template <uint32_t NW, bool ST>
__global__ void __launch_bounds__(64 * NW) reg(const uint8_t *__restrict__ recs, const uint32_t *__restrict__ offs, uint64_t n,
                                               uint64_t wtpb, uint32_t *out, uint32_t *log)
{
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t nwt = (n + WT - 1) / WT, last = n - 1;
    const uint64_t wbeg = blockIdx.x * wtpb, wend = min(wbeg + wtpb, nwt);
    const uint32_t ntl = wend > wbeg + wave ? (uint32_t)((wend - wbeg - wave + NW - 1) / NW) : 0u;
    auto tile_of = [&](uint32_t k) -> uint64_t { return wbeg + wave + (uint64_t)NW * min(k, ntl - 1); };
    auto off_of = [&](uint32_t k) -> uint32_t { return offs[min<uint64_t>(tile_of(k) * WT + lane, last)]; };
    auto wl = [&](uint32_t off, uint4 (&W)[5]) {
        const uint4 *p = reinterpret_cast<const uint4 *>(recs + (off & ~3u));
#pragma unroll
        for (int j = 0; j < 5; j++) W[j] = p[j];
    };
    uint32_t acc = 0;
    auto tile = [&](uint32_t k, uint32_t off, const uint4 (&W)[5]) {
        const uint64_t i = tile_of(k) * WT + lane;
        const uint32_t a = fold(W, off & 3);
        acc += a;
        if (ST && i < n) log[i] = a;
    };
    uint4 WA[5], WB[5];
    uint32_t oA = 0, oB = 0;
    if (ntl) {
        oA = off_of(0);
        oB = off_of(1);
        wl(oA, WA);
    }
    for (uint32_t k = 0; k < ntl; k += 2) {
        const uint32_t oN = off_of(k + 2);
        wl(oB, WB);
        tile(k, oA, WA);
        if (k + 1 >= ntl) break;
        const uint32_t oN2 = off_of(k + 3);
        wl(oN, WA);
        oA = oN;
        tile(k + 1, oB, WB);
        oB = oN2;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// per-wave LDS ring: Q tile slots of NJ KiB, offset rows (lane starts + tile end) 2Q tiles ahead
template <int Q, int NJ>
struct RingWave {
    uint4 slot[Q][NJ * 64];
    uint32_t lo[2 * Q + 1][64];
    uint32_t hi[2 * Q + 1][64];
};
// SM (IP-log store mode): 0 none, 1 a 4-B store per lane per tile, 2 the same non-temporal,
// 3 batched: the wave's four consecutive tiles (MAP 1: super-tiles of four contiguous tiles per
// wave) staged in LDS and written as one 16-B store per lane
template <uint32_t NW, int Q, int NJ, int SM, int MAP = 0>
__global__ void __launch_bounds__(64 * NW) ring(const uint8_t *__restrict__ recs, const uint32_t *__restrict__ offs, uint64_t n,
                                                uint64_t wtpb, uint32_t *out, uint32_t *log)
{
    constexpr int R = 2 * Q + 1;                  // offset rows
    constexpr int STP = (SM == 1 || SM == 2 || SM == 4) ? 1 : 0; // stores per step counted exactly
    constexpr int OPS = NJ + 2 + STP;             // vector-memory ops one step issues (SM 3: stores not counted)
    __shared__ RingWave<Q, NJ> RW[NW];
    __shared__ uint32_t stage[NW][4 * 64];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    RingWave<Q, NJ> &W = RW[wave];
    const uint64_t nwt = (n + WT - 1) / WT;
    const uint64_t wbeg = blockIdx.x * wtpb, wend = min(wbeg + wtpb, nwt);
    uint32_t ntl;
    if (MAP == 0) ntl = wend > wbeg + wave ? (uint32_t)((wend - wbeg - wave + NW - 1) / NW) : 0u;
    else {
        // super-tiles of 4 tiles: wave w takes super-tiles w, w + NW, ... (the range holds whole ones)
        const uint64_t nst = wend > wbeg ? (wend - wbeg) / 4 : 0;
        ntl = nst > wave ? (uint32_t)(4 * ((nst - wave + NW - 1) / NW)) : 0u;
    }
    if (!ntl) return;
    auto tile_of = [&](int64_t k) -> uint64_t {
        const uint64_t kk = (uint64_t)min<int64_t>(max<int64_t>(k, 0), ntl - 1);
        return MAP == 0 ? wbeg + wave + (uint64_t)NW * kk : wbeg + 4 * (wave + (uint64_t)NW * (kk / 4)) + kk % 4;
    };
    // offs has n + 1 entries (the last: the blob's end)
    auto rows = [&](int64_t k) {
        const uint64_t r = tile_of(k) * WT + lane;
        const uint32_t row = (uint32_t)(k % R);
        dma4(offs + min<uint64_t>(r, n), lds_addr(&W.lo[row][0]));
        dma4(offs + min<uint64_t>(tile_of(k) * WT + WT, n), lds_addr(&W.hi[row][0]));
    };
    auto pieces = [&](int64_t k) {
        const uint32_t row = (uint32_t)(k % R);
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(W.lo[row][0]);
        const uint32_t b1 = __builtin_amdgcn_readfirstlane(W.hi[row][0]);
        const uint32_t base = b0 & ~15u, nch = (b1 - base + 15) >> 4;
        const uint32_t dst = lds_addr(&W.slot[k % Q][0]);
#pragma unroll
        for (int j = 0; j < NJ; j++) dma16(recs + base + min((uint32_t)(j * 64) + lane, nch - 1) * 16, dst + j * 1024);
    };
    const uint64_t scratch = n + (blockIdx.x * NW + wave) * 64 + lane;
    for (int k = 0; k <= Q; k++) rows(k);
    vmcnt<0>();
    for (int k = 1 - Q; k < 0; k++) {
        rows(k + 2 * Q);
        pieces(k + Q - 1);
        if (STP) log[scratch] = 0; // keep the op count of a step
    }
    uint32_t acc = 0;
    for (uint32_t k = 0; k < ntl; k++) {
        rows((int64_t)k + 2 * Q);
        vmcnt<(NJ + STP + Q * OPS + 2 < 63 ? NJ + STP + Q * OPS + 2 : 63)>();
        pieces((int64_t)k + Q - 1);
        vmcnt<(Q - 1) * OPS>(); // tile k landed
        const uint32_t row = k % R;
        const uint32_t off = W.lo[row][lane];
        const uint32_t base = __builtin_amdgcn_readfirstlane(W.lo[row][0]) & ~15u;
        const uint32_t rel = off - base;
        const uint4 *q = &W.slot[k % Q][rel >> 4];
        uint4 V[5];
#pragma unroll
        for (int j = 0; j < 5; j++) V[j] = q[j];
        const uint32_t a = fold(V, 0) ^ (rel & 15); // records of this probe are 16-B aligned
        acc += a;
        const uint64_t i = tile_of(k) * WT + lane;
        if (SM == 1) log[i < n ? i : scratch] = a;
        if (SM == 2) __builtin_nontemporal_store(a, &log[i < n ? i : scratch]);
        if (SM == 4) log[i & 0x3ffff] = a; // an L2-resident 1-MiB target: HBM writes or the store itself?
        if (SM == 3) {
            stage[wave][(k & 3) * 64 + lane] = a;
            if ((k & 3) == 3) {
                const uint4 v = reinterpret_cast<const uint4 *>(stage[wave])[lane];
                const uint64_t j = tile_of(k - 3) * WT + 4 * lane;
                *reinterpret_cast<uint4 *>(&log[j + 4 <= n ? j : (scratch & ~3ull)]) = v;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// SM 5: the IP-log stores leave from a writer wave (wave NW of the workgroup): each parse wave
// puts its tile's values in an LDS ring of S tiles and publishes a count; the writer drains the
// rings with 4-B stores, so no parse wave's vmcnt wait ever covers a store
template <uint32_t NW, int Q, int NJ, int S>
__global__ void __launch_bounds__(64 * (NW + 1)) ringw(const uint8_t *__restrict__ recs, const uint32_t *__restrict__ offs,
                                                      uint64_t n, uint64_t wtpb, uint32_t *out, uint32_t *log)
{
    constexpr int R = 2 * Q + 1;
    constexpr int OPS = NJ + 2;
    __shared__ RingWave<Q, NJ> RW[NW];
    __shared__ uint32_t stage[NW][S][64];
    __shared__ uint32_t prod[NW], cons[NW];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (threadIdx.x < NW) { prod[threadIdx.x] = 0; cons[threadIdx.x] = 0; }
    __syncthreads();
    const uint64_t nwt = (n + WT - 1) / WT;
    const uint64_t wbeg = blockIdx.x * wtpb, wend = min(wbeg + wtpb, nwt);
    auto ntl_of = [&](uint32_t w) -> uint32_t { return wend > wbeg + w ? (uint32_t)((wend - wbeg - w + NW - 1) / NW) : 0u; };
    if (wave == NW) {
        // writer
        uint32_t done[NW];
        uint32_t nt[NW];
        for (uint32_t w = 0; w < NW; w++) { done[w] = 0; nt[w] = ntl_of(w); }
        for (;;) {
            bool left = false, moved = false;
            for (uint32_t w = 0; w < NW; w++) {
                if (done[w] >= nt[w]) continue;
                left = true;
                const uint32_t p = __hip_atomic_load(&prod[w], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                while (done[w] < p) {
                    const uint32_t v = stage[w][done[w] % S][lane];
                    const uint64_t i = (wbeg + w + (uint64_t)NW * done[w]) * WT + lane;
                    if (i < n) log[i] = v;
                    done[w]++;
                    moved = true;
                }
                if (lane == 0) __hip_atomic_store(&cons[w], done[w], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (!left) break;
            if (!moved) __builtin_amdgcn_s_sleep(2);
        }
        return;
    }
    RingWave<Q, NJ> &W = RW[wave];
    const uint32_t ntl = ntl_of(wave);
    if (!ntl) return;
    auto tile_of = [&](int64_t k) -> uint64_t { return wbeg + wave + (uint64_t)NW * (uint64_t)min<int64_t>(max<int64_t>(k, 0), ntl - 1); };
    auto rows = [&](int64_t k) {
        const uint64_t r = tile_of(k) * WT + lane;
        const uint32_t row = (uint32_t)(k % R);
        dma4(offs + min<uint64_t>(r, n), lds_addr(&W.lo[row][0]));
        dma4(offs + min<uint64_t>(tile_of(k) * WT + WT, n), lds_addr(&W.hi[row][0]));
    };
    auto pieces = [&](int64_t k) {
        const uint32_t row = (uint32_t)(k % R);
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(W.lo[row][0]);
        const uint32_t b1 = __builtin_amdgcn_readfirstlane(W.hi[row][0]);
        const uint32_t base = b0 & ~15u, nch = (b1 - base + 15) >> 4;
        const uint32_t dst = lds_addr(&W.slot[k % Q][0]);
#pragma unroll
        for (int j = 0; j < NJ; j++) dma16(recs + base + min((uint32_t)(j * 64) + lane, nch - 1) * 16, dst + j * 1024);
    };
    for (int k = 0; k <= Q; k++) rows(k);
    vmcnt<0>();
    for (int k = 1 - Q; k < 0; k++) {
        rows(k + 2 * Q);
        pieces(k + Q - 1);
    }
    uint32_t acc = 0;
    for (uint32_t k = 0; k < ntl; k++) {
        rows((int64_t)k + 2 * Q);
        vmcnt<(NJ + Q * OPS + 2 < 63 ? NJ + Q * OPS + 2 : 63)>();
        pieces((int64_t)k + Q - 1);
        vmcnt<(Q - 1) * OPS>();
        const uint32_t row = k % R;
        const uint32_t off = W.lo[row][lane];
        const uint32_t base = __builtin_amdgcn_readfirstlane(W.lo[row][0]) & ~15u;
        const uint32_t rel = off - base;
        const uint4 *q = &W.slot[k % Q][rel >> 4];
        uint4 V[5];
#pragma unroll
        for (int j = 0; j < 5; j++) V[j] = q[j];
        const uint32_t a = fold(V, 0) ^ (rel & 15);
        acc += a;
        while (__hip_atomic_load(&cons[wave], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) + S <= k) __builtin_amdgcn_s_sleep(1);
        stage[wave][k % S][lane] = a;
        if (lane == 0) __hip_atomic_store(&prod[wave], k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
    const size_t bytes = n * REC + 256;
    uint8_t *d;
    uint32_t *o, *offs, *log;
    hipMalloc(&d, bytes);
    hipMalloc(&o, 4);
    hipMalloc(&offs, (n + 1) * 4);
    hipMalloc(&log, (n + (1 << 22)) * 4);
    hipMemset(d, 1, bytes);
    std::vector<uint32_t> h(n + 1);
    for (uint64_t i = 0; i <= n; i++) h[i] = (uint32_t)(i * REC);
    hipMemcpy(offs, h.data(), (n + 1) * 4, hipMemcpyHostToDevice);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint64_t nwt = (n + WT - 1) / WT;
    auto timeit = [&](const char *name, int wgcu, auto launch) {
        float best = 1e9f, sum = 0;
        for (int it = 0; it < 12; it++) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (it >= 2) { sum += ms; if (ms < best) best = ms; }
        }
        hipError_t e = hipGetLastError();
        printf("%-26s wg/cu=%d  best %.1f us  mean %.1f us  %.0f GB/s  %s\n", name, wgcu, best * 1e3, sum / 10 * 1e3,
               n * (double)REC / (best * 1e-3) / 1e9, e == hipSuccess ? "" : hipGetErrorString(e));
        fflush(stdout);
    };
    for (int wgcu : {2, 4, 8}) {
        const uint64_t grid = (uint64_t)cus * wgcu;
        timeit("plain", wgcu, [&] { hipLaunchKernelGGL(plain, dim3(grid), dim3(256), 0, 0, (const uint4 *)d, n * REC / 16, o); });
    }
#define RUN(NAME, KERNEL, NW)                                                                                  \
    for (int wgcu : {1, 2}) {                                                                                  \
        const uint64_t grid = (uint64_t)cus * wgcu, wtpb = (nwt + grid - 1) / grid;                            \
        timeit(NAME, wgcu, [&] { hipLaunchKernelGGL(KERNEL, dim3(grid), dim3(64 * NW), 0, 0, d, offs, n, wtpb, o, log); }); \
    }
    RUN("ring Q4 NJ6", (ring<4, 4, 6, 0>), 4);
    RUN("ring Q4 NJ6 st4", (ring<4, 4, 6, 1>), 4);
    for (int wgcu : {1, 2}) {
        const uint64_t grid = (uint64_t)cus * wgcu, wtpb = (nwt + grid - 1) / grid;
        timeit("ringw Q4 NJ6 S8", wgcu, [&] { hipLaunchKernelGGL((ringw<4, 4, 6, 8>), dim3(grid), dim3(64 * 5), 0, 0, d, offs, n, wtpb, o, log); });
        timeit("ringw Q4 NJ6 S16", wgcu, [&] { hipLaunchKernelGGL((ringw<4, 4, 6, 16>), dim3(grid), dim3(64 * 5), 0, 0, d, offs, n, wtpb, o, log); });
    }
    return 0;
}
