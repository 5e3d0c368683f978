// tools/sort_probe.hip — the transaction stage's key sort alone (pv_radix_sort_pairs: 64-bit keys
// (hash31 << 32 | rank), 32-bit values), rocPRIM onesweep at 7, 8 and 9 bits per pass and over the
// key bits in use, against the default. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/sort_probe tools/sort_probe.hip
//   tools/sort_probe [n]
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

template <unsigned Bits, unsigned Block = 256>
using OneCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                          rocprim::radix_sort_onesweep_config<rocprim::kernel_config<Block, 12>,
                                                                              rocprim::kernel_config<Block, 12>, Bits>>;

template <class Cfg>
static float run(const char *name, uint64_t *kin, uint64_t *kout, uint32_t *vin, uint32_t *vout, size_t n, int b0, int b1,
                 const std::vector<uint64_t> &want)
{
    size_t tmp = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tmp, kin, kout, vin, vout, n, b0, b1, 0));
    void *d_tmp;
    CK(hipMalloc(&d_tmp, tmp));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++) CK(rocprim::radix_sort_pairs<Cfg>(d_tmp, tmp, kin, kout, vin, vout, n, b0, b1, 0));
    const int it = 20;
    CK(hipEventRecord(a, 0));
    for (int k = 0; k < it; k++) CK(rocprim::radix_sort_pairs<Cfg>(d_tmp, tmp, kin, kout, vin, vout, n, b0, b1, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint64_t> got(n);
    CK(hipMemcpy(got.data(), kout, n * 8, hipMemcpyDeviceToHost));
    const bool ok = got == want;
    printf("%-28s bits [%d,%d) %8.1f us %s\n", name, b0, b1, 1000.0f * ms / it, ok ? "ok" : "MISMATCH");
    CK(hipFree(d_tmp));
    return ms / it;
}


// ---- bucket sort: count by the top B key bits (bit 63, the sentinel, its own last bucket),
// scan, scatter, then each bucket sorted on its own
__device__ __forceinline__ uint32_t bucket_of(uint64_t k, uint32_t B)
{
    return (k >> 63) ? (1u << B) : (uint32_t)(k >> (63 - B));
}
__global__ void __launch_bounds__(256) xs_count(const uint64_t *k, size_t n, uint32_t B, uint32_t *cnt)
{
    extern __shared__ uint32_t h[];
    const uint32_t nb = (1u << B) + 1;
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) h[j] = 0;
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        atomicAdd(&h[bucket_of(k[i], B)], 1u);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x)
        if (h[j]) atomicAdd(&cnt[j], h[j]);
}
// exclusive scan of nb counts (one workgroup of 1024 threads): off[0..nb], cur = off
__global__ void __launch_bounds__(1024) xs_scan(const uint32_t *cnt, uint32_t nb, uint32_t *off, uint32_t *cur)
{
    __shared__ uint32_t part[1024];
    const uint32_t per = (nb + 1023) / 1024, a = threadIdx.x * per, b = min(a + per, nb);
    uint32_t s = 0;
    for (uint32_t j = a; j < b; j++) s += cnt[j];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0u;
    for (uint32_t j = a; j < b; j++) { off[j] = run; cur[j] = run; run += cnt[j]; }
    if (threadIdx.x == 1023) off[nb] = part[1023];
}
__global__ void __launch_bounds__(256) xs_scatter(const uint64_t *k, const uint32_t *v, size_t n, uint32_t B, uint32_t *cur,
                                                  uint64_t *ko, uint32_t *vo)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t x = k[i];
        const uint32_t p = atomicAdd(&cur[bucket_of(x, B)], 1u);
        ko[p] = x;
        vo[p] = v[i];
    }
}
// one bucket per workgroup, bitonic in LDS (buckets up to XS_CAP; timing only, no fallback)
#define XS_CAP 4096
__global__ void __launch_bounds__(512) xs_local(const uint64_t *k, const uint32_t *v, const uint32_t *off, uint32_t nbk,
                                                uint64_t *ko, uint32_t *vo)
{
    __shared__ uint64_t sk[XS_CAP];
    __shared__ uint32_t sv[XS_CAP];
    const uint32_t b = blockIdx.x;
    const uint32_t a = off[b], s = off[b + 1] - a;
    if (b >= nbk || s == 0) return;
    uint32_t P = 1;
    while (P < s) P <<= 1;
    if (P > XS_CAP) return;
    for (uint32_t j = threadIdx.x; j < P; j += blockDim.x) {
        sk[j] = j < s ? k[a + j] : ~0ull;
        sv[j] = j < s ? v[a + j] : 0u;
    }
    __syncthreads();
    for (uint32_t len = 2; len <= P; len <<= 1)
        for (uint32_t st = len >> 1; st > 0; st >>= 1) {
            for (uint32_t t = threadIdx.x; t < P / 2; t += blockDim.x) {
                const uint32_t i = 2 * st * (t / st) + (t % st), j = i + st;
                const bool up = (i & len) == 0;
                const uint64_t x = sk[i], y = sk[j];
                if ((x > y) == up) {
                    sk[i] = y; sk[j] = x;
                    const uint32_t w = sv[i]; sv[i] = sv[j]; sv[j] = w;
                }
            }
            __syncthreads();
        }
    for (uint32_t j = threadIdx.x; j < s; j += blockDim.x) {
        ko[a + j] = sk[j];
        vo[a + j] = sv[j];
    }
}

static float run_bucket(const char *name, bool seg, uint64_t *kin, uint64_t *kout, uint32_t *vin, uint32_t *vout, size_t n,
                        const std::vector<uint64_t> &want)
{
    uint32_t B = 4;
    while (B < 14 && (n >> B) > 768) B++;
    const uint32_t nb = (1u << B) + 1;
    uint32_t *cnt, *off, *cur;
    uint64_t *kt;
    uint32_t *vt;
    CK(hipMalloc(&cnt, nb * 4));
    CK(hipMalloc(&off, (nb + 1) * 4));
    CK(hipMalloc(&cur, nb * 4));
    CK(hipMalloc(&kt, n * 8));
    CK(hipMalloc(&vt, n * 4));
    size_t tmp = 0;
    void *d_tmp = nullptr;
    if (seg) {
        CK(rocprim::segmented_radix_sort_pairs(nullptr, tmp, kt, kout, vt, vout, n, 1u << B, off, off + 1, 0, 63, 0));
        CK(hipMalloc(&d_tmp, tmp));
    }
    const uint32_t grid = (uint32_t)std::min<size_t>(2048, (n + 4095) / 4096 + 1);
    auto once = [&]() {
        CK(hipMemsetAsync(cnt, 0, nb * 4, 0));
        hipLaunchKernelGGL(xs_count, dim3(grid), dim3(256), nb * 4, 0, kin, n, B, cnt);
        hipLaunchKernelGGL(xs_scan, dim3(1), dim3(1024), 0, 0, cnt, nb, off, cur);
        hipLaunchKernelGGL(xs_scatter, dim3(grid), dim3(256), 0, 0, kin, vin, n, B, cur, kt, vt);
        if (seg) CK(rocprim::segmented_radix_sort_pairs(d_tmp, tmp, kt, kout, vt, vout, n, 1u << B, off, off + 1, 0, 63, 0));
        else hipLaunchKernelGGL(xs_local, dim3(nb), dim3(512), 0, 0, kt, vt, off, 1u << B, kout, vout);
    };
    for (int w = 0; w < 3; w++) once();
    {
        // phase times of one run
        hipEvent_t ev[6];
        for (auto &e : ev) CK(hipEventCreate(&e));
        CK(hipEventRecord(ev[0], 0));
        CK(hipMemsetAsync(cnt, 0, nb * 4, 0));
        hipLaunchKernelGGL(xs_count, dim3(grid), dim3(256), nb * 4, 0, kin, n, B, cnt);
        CK(hipEventRecord(ev[1], 0));
        hipLaunchKernelGGL(xs_scan, dim3(1), dim3(1024), 0, 0, cnt, nb, off, cur);
        CK(hipEventRecord(ev[2], 0));
        hipLaunchKernelGGL(xs_scatter, dim3(grid), dim3(256), 0, 0, kin, vin, n, B, cur, kt, vt);
        CK(hipEventRecord(ev[3], 0));
        if (seg) CK(rocprim::segmented_radix_sort_pairs(d_tmp, tmp, kt, kout, vt, vout, n, 1u << B, off, off + 1, 0, 63, 0));
        else hipLaunchKernelGGL(xs_local, dim3(nb), dim3(512), 0, 0, kt, vt, off, 1u << B, kout, vout);
        CK(hipEventRecord(ev[4], 0));
        CK(hipEventSynchronize(ev[4]));
        float t[4];
        for (int q = 0; q < 4; q++) CK(hipEventElapsedTime(&t[q], ev[q], ev[q + 1]));
        printf("  phases: count %.1f scan %.1f scatter %.1f local %.1f us\n", 1000 * t[0], 1000 * t[1], 1000 * t[2], 1000 * t[3]);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int it = 20;
    CK(hipEventRecord(a, 0));
    for (int k = 0; k < it; k++) once();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint64_t> got(n);
    CK(hipMemcpy(got.data(), kout, n * 8, hipMemcpyDeviceToHost));
    // the sentinel bucket is not sorted (all keys equal): compare the rest
    const bool ok = got == want;
    printf("%-28s B=%u %8.1f us %s\n", name, B, 1000.0f * ms / it, ok ? "ok" : "MISMATCH");
    CK(hipFree(cnt)); CK(hipFree(off)); CK(hipFree(cur)); CK(hipFree(kt)); CK(hipFree(vt));
    if (d_tmp) CK(hipFree(d_tmp));
    return ms / it;
}

int main(int argc, char **argv)
{
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 3000000;
    std::mt19937_64 rng(7);
    std::vector<uint64_t> k(n);
    std::vector<uint32_t> v(n);
    for (size_t i = 0; i < n; i++) {
        const uint64_t h = (rng() >> 33) & 0x7fffffffull;                 // hash31
        k[i] = (h << 32) | (uint32_t)(4 * ((i * 2654435761ull) % n)); // ranks in scrambled order
        v[i] = (uint32_t)i;
    }
    std::vector<uint64_t> want = k;
    std::sort(want.begin(), want.end());
    uint64_t *kin, *kout;
    uint32_t *vin, *vout;
    CK(hipMalloc(&kin, n * 8));
    CK(hipMalloc(&kout, n * 8));
    CK(hipMalloc(&vin, n * 4));
    CK(hipMalloc(&vout, n * 4));
    CK(hipMemcpy(kin, k.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(vin, v.data(), n * 4, hipMemcpyHostToDevice));
    printf("n = %zu\n", n);
    run<rocprim::default_config>("default", kin, kout, vin, vout, n, 0, 64, want);
    run<rocprim::default_config>("default", kin, kout, vin, vout, n, 0, 63, want);
    run<OneCfg<8>>("onesweep 8", kin, kout, vin, vout, n, 0, 63, want);
    run<OneCfg<9, 128>>("onesweep 9 (128)", kin, kout, vin, vout, n, 0, 63, want);
    run<OneCfg<7>>("onesweep 7", kin, kout, vin, vout, n, 0, 63, want);
    run_bucket("bucket + LDS bitonic", false, kin, kout, vin, vout, n, want);
    run_bucket("bucket + rocprim segmented", true, kin, kout, vin, vout, n, want);
    // hash in 24 bits above a 32-bit rank: 56 bits
    std::vector<uint64_t> k56(n);
    for (size_t i = 0; i < n; i++) k56[i] = ((k[i] >> 39) << 32) | (uint32_t)k[i];
    std::vector<uint64_t> w56 = k56;
    std::sort(w56.begin(), w56.end());
    CK(hipMemcpy(kin, k56.data(), n * 8, hipMemcpyHostToDevice));
    run<rocprim::default_config>("default hash24", kin, kout, vin, vout, n, 0, 56, w56);
    run<OneCfg<8>>("onesweep 8 hash24", kin, kout, vin, vout, n, 0, 56, w56);
    run<OneCfg<7>>("onesweep 7 hash24", kin, kout, vin, vout, n, 0, 56, w56);
    return 0;
}
