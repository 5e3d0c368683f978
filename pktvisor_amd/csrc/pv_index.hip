// SPDX-License-Identifier: MPL-2.0
//
// pv_index.hip — the pcap record index on the device, for the host-memory ingest path.
//
// The reference walks a capture one record at a time (PcapInputStream::_open_pcap,
// src/inputs/pcap/PcapInputStream.cpp:471-527). pv_index_records is that walk on the host;
// here it runs on the chunk the ingest has just copied to HBM, so the host only copies.
// The chunk is cut into PV_IX_SEG-byte segments, one lane each:
//
//   1. pv_ix_guess: segment 0 starts at the first record (X.first); segment s > 0 guesses its first record
//      start (the first offset from which four headers are plausible, as the host's
//      parallel index guesses) and walks to its end: records starting in the segment,
//      and the position after them (its exit).
//   2. pv_ix_fix, repeated until nothing changes: the true first start of segment s is
//      segment s - 1's exit; a segment whose guess differs walks again from there.
//      Exits are double-buffered, so one pass moves the validated chain on by at least
//      one segment and a correct guess settles in one pass.
//   3. pv_ix_scan: record counts to per-segment bases (one workgroup).
//   4. pv_ix_write: each segment writes its record offsets.
//   5. pv_ix_secs: the ts_sec change points and monotonicity, one lane per record.
//
// Walks are deterministic and the chain is validated from byte 0, so the offsets equal the
// sequential walk's for any input; the guesses only decide how many fix passes run.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pv_layout.h"

#define PV_IX_BACK 4096u // segments a fix pass looks back over for an exit (8 MiB)



namespace {

__device__ __forceinline__ void hdr(const uint8_t *r, uint64_t p, uint32_t &sec, uint32_t &frac, uint32_t &cl, uint32_t &len)
{
    // record headers are 4-byte aligned only when every caplen is: byte loads in general
    const uint8_t *h = r + p;
    if ((p & 3) == 0) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(h);
        sec = w[0]; frac = w[1]; cl = w[2]; len = w[3];
        return;
    }
    uint32_t w[4];
    for (int k = 0; k < 4; k++)
        w[k] = (uint32_t)h[4 * k] | ((uint32_t)h[4 * k + 1] << 8) | ((uint32_t)h[4 * k + 2] << 16) | ((uint32_t)h[4 * k + 3] << 24);
    sec = w[0]; frac = w[1]; cl = w[2]; len = w[3];
}
__device__ __forceinline__ uint32_t caplen_at(const uint8_t *r, uint64_t p)
{
    const uint8_t *h = r + p + 8;
    if ((p & 3) == 0) return *reinterpret_cast<const uint32_t *>(h);
    return (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
}

// the host's plausibility test (pv_ingest.cpp plausible): four headers with ts_sec within a
// day of the chunk's first, the sub-second field in range, caplen <= min(len, 256 KiB)
__device__ bool plausible(const PvIxParams &X, uint64_t p)
{
    for (int k = 0; k < 4; k++) {
        if (p == X.bytes) return true;
        if (p + 16 > X.bytes) return k > 0;
        uint32_t sec, frac, cl, len;
        hdr(X.recs, p, sec, frac, cl, len);
        const uint32_t dsec = sec > X.sec0 ? sec - X.sec0 : X.sec0 - sec;
        if (dsec > 86400 || cl > (256u << 10) || cl > len || frac >= X.frac_lim) return false;
        if (p + 16 + (uint64_t)cl > X.bytes) return k > 0;
        p += 16 + (uint64_t)cl;
    }
    return true;
}

// records starting in [p, hi) from p: their count and the position after them
__device__ uint64_t walk(const PvIxParams &X, uint64_t p, uint64_t hi, uint32_t &n)
{
    n = 0;
    while (p < hi) {
        if (p + 16 > X.bytes) return p | PV_IX_STOP;
        const uint32_t cl = caplen_at(X.recs, p);
        if (p + 16 + (uint64_t)cl > X.bytes) return p | PV_IX_STOP;
        n++;
        p += 16 + (uint64_t)cl;
    }
    return p;
}

__device__ __forceinline__ uint64_t seg_lo(const PvIxParams &X, uint32_t s) { return (uint64_t)s * PV_IX_SEG; }
__device__ __forceinline__ uint64_t seg_hi(const PvIxParams &X, uint32_t s) { return min<uint64_t>(X.bytes, (uint64_t)(s + 1) * PV_IX_SEG); }

} // namespace

// pv_ix_guess stages its segment, and the first header past it, in LDS: one wave per segment
#define PV_IX_WIN (PV_IX_SEG + 64)
#define PV_IX_WAVES 4

namespace {

// 16 bytes at byte o of a staged segment, as four little-endian words (five aligned LDS
// reads and byte alignment, not sixteen byte reads)
__device__ __forceinline__ void win_hdr(const uint32_t *w, uint32_t o, uint32_t &sec, uint32_t &frac, uint32_t &cl,
                                        uint32_t &len)
{
    const uint32_t a = o >> 2, sh = o & 3;
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++) d[k] = w[a + k];
    sec = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
    frac = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
    cl = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
    len = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
}
__device__ __forceinline__ uint32_t win_caplen(const uint32_t *w, uint32_t o)
{
    const uint32_t a = (o + 8) >> 2, sh = (o + 8) & 3;
    return __builtin_amdgcn_alignbyte(w[a + 1], w[a], sh);
}

// plausible() with the headers inside the staged window [lo, lo + PV_IX_WIN) read from LDS
__device__ bool plausible_w(const PvIxParams &X, const uint32_t *w, uint64_t lo, uint64_t p)
{
    for (int k = 0; k < 4; k++) {
        if (p == X.bytes) return true;
        if (p + 16 > X.bytes) return k > 0;
        uint32_t sec, frac, cl, len;
        if (p + 20 <= lo + PV_IX_WIN) win_hdr(w, (uint32_t)(p - lo), sec, frac, cl, len);
        else hdr(X.recs, p, sec, frac, cl, len);
        const uint32_t dsec = sec > X.sec0 ? sec - X.sec0 : X.sec0 - sec;
        if (dsec > 86400 || cl > (256u << 10) || cl > len || frac >= X.frac_lim) return false;
        if (p + 16 + (uint64_t)cl > X.bytes) return k > 0;
        p += 16 + (uint64_t)cl;
    }
    return true;
}

// walk() with the caplens inside the staged window read from LDS
__device__ uint64_t walk_w(const PvIxParams &X, const uint32_t *w, uint64_t lo, uint64_t p, uint64_t hi, uint32_t &n)
{
    n = 0;
    while (p < hi) {
        if (p + 16 > X.bytes) return p | PV_IX_STOP;
        const uint32_t cl = p + 16 <= lo + PV_IX_WIN ? win_caplen(w, (uint32_t)(p - lo)) : caplen_at(X.recs, p);
        if (p + 16 + (uint64_t)cl > X.bytes) return p | PV_IX_STOP;
        n++;
        p += 16 + (uint64_t)cl;
    }
    return p;
}

} // namespace

// One wave per segment: the segment is staged in LDS with 16-B loads, the lanes test 64
// consecutive candidate offsets per round (the first plausible one by ballot, so the guess is
// the sequential scan's), and lane 0 walks the segment from LDS. A record start lies within
// the first record length of the segment, so a round or a few settle the guess.
extern "C" __global__ void __launch_bounds__(64 * PV_IX_WAVES) pv_ix_guess(const PvIxParams *__restrict__ Xp)
{
    const PvIxParams X = *Xp;
    __shared__ uint4 win[PV_IX_WAVES][PV_IX_WIN / 16 + 1]; // + 1: win_hdr's fifth word
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const uint32_t s = blockIdx.x * PV_IX_WAVES + wv;
    const bool live = s < X.nseg;
    const uint64_t lo = seg_lo(X, s);
    constexpr uint32_t NQ = PV_IX_WIN / 16, QR = (NQ + 63) / 64;
    if (live) {
        // bytes past X.bytes are staged as they lie (the buffer's pad); every test is bounded by X.bytes
        uint4 v[QR];
#pragma unroll
        for (uint32_t u = 0; u < QR; u++) {
            const uint32_t q = ln + u * 64;
            if (q < NQ && lo + q * 16 < X.bytes) v[u] = *reinterpret_cast<const uint4 *>(X.recs + lo + q * 16);
        }
#pragma unroll
        for (uint32_t u = 0; u < QR; u++) {
            const uint32_t q = ln + u * 64;
            if (q < NQ && lo + q * 16 < X.bytes) win[wv][q] = v[u];
        }
    }
    __syncthreads();
    if (!live) return;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(win[wv]);
    const uint64_t hi = seg_hi(X, s);
    uint64_t p = X.first;
    if (s > 0) {
        p = PV_IX_NONE;
        for (uint64_t b = lo; b < hi; b += 64) {
            const uint64_t q = b + ln;
            const uint64_t m = __ballot(q < hi && plausible_w(X, w, lo, q));
            if (m) { p = b + __builtin_ctzll(m); break; }
        }
        if (p == PV_IX_NONE) {
            if (ln == 0) {
                X.start[s] = PV_IX_NONE;
                X.cnt[s] = 0;
                X.exit[0][s] = PV_IX_NONE;
            }
            return;
        }
    }
    if (ln == 0) {
        uint32_t n;
        X.start[s] = p;
        X.exit[0][s] = walk_w(X, w, lo, p, hi, n);
        X.cnt[s] = n;
    }
}

// one validation pass: exit[src] -> exit[src ^ 1]
extern "C" __global__ void pv_ix_fix(const PvIxParams *__restrict__ Xp, uint32_t src)
{
    const PvIxParams X = *Xp;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= X.nseg) return;
    const uint64_t *ein = X.exit[src];
    uint64_t *eout = X.exit[src ^ 1];
    if (s == 0) { eout[0] = ein[0]; return; }
    // the exit of the nearest earlier segment that has one: segments with no start of their
    // own (inside a long record) are skipped, so a record spanning many segments settles in
    // one pass instead of one segment per pass
    uint32_t t = s - 1;
    while (t > 0 && ein[t] == PV_IX_NONE && s - t < PV_IX_BACK) t--;
    const uint64_t prev = ein[t];
    uint64_t cur = ein[s];
    // the chain has not reached here yet, or lands in a skipped segment that walks first
    if (prev == PV_IX_NONE || (!(prev & PV_IX_STOP) && prev < seg_lo(X, s))) { eout[s] = cur; return; }
    const uint64_t hi = seg_hi(X, s);
    if (prev & PV_IX_STOP) {
        // the walk stopped before this segment: no records here
        if (X.start[s] != prev || cur != prev) {
            X.start[s] = prev;
            X.cnt[s] = 0;
            cur = prev;
            atomicOr(&X.status[0], 1u);
        }
    } else if (prev >= hi) {
        // a record spans this whole segment
        if (X.start[s] != prev || cur != prev) {
            X.start[s] = prev;
            X.cnt[s] = 0;
            cur = prev;
            atomicOr(&X.status[0], 1u);
        }
    } else if (X.start[s] != prev) {
        uint32_t n;
        X.start[s] = prev;
        cur = walk(X, prev, hi, n);
        X.cnt[s] = n;
        atomicOr(&X.status[0], 1u);
    }
    eout[s] = cur;
}

// exclusive prefix of the segment counts (one workgroup of 1024): tiles of 8192 counts staged
// in LDS with coalesced loads, each thread summing eight consecutive counts, a wave-shuffle scan
// of the sums, and coalesced stores of the bases
extern "C" __global__ void __launch_bounds__(1024) pv_ix_scan(const PvIxParams *__restrict__ Xp)
{
    const PvIxParams X = *Xp;
    constexpr uint32_t PER = 8, T = PER * 1024;
    __shared__ uint32_t tile[T + T / 32]; // one pad word per 32: a thread's eight counts are not all in one bank
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x, ln = t & 63, wv = t >> 6;
    auto at = [](uint32_t i) { return i + i / 32; };
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < X.nseg; t0 += T) {
        uint32_t v[PER];
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) {
            const uint32_t i = t0 + u * 1024 + t;
            v[u] = i < X.nseg ? X.cnt[i] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) tile[at(u * 1024 + t)] = v[u];
        __syncthreads();
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) { v[u] = tile[at(t * PER + u)]; sum += v[u]; }
        uint32_t x = sum;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (ln >= o) x += y;
        }
        if (ln == 63) ws[wv] = x;
        __syncthreads();
        uint32_t run = carry + x - sum, total = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
            const uint32_t z = ws[k];
            if (k < wv) run += z;
            total += z;
        }
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) { tile[at(t * PER + u)] = run; run += v[u]; }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < PER; u++) {
            const uint32_t i = t0 + u * 1024 + t;
            if (i < X.nseg) X.base[i] = tile[at(u * 1024 + t)];
        }
        carry += total;
        __syncthreads(); // tile and ws are the next tile's
    }
    if (t == 0) X.base[X.nseg] = carry;
}

extern "C" __global__ void pv_ix_write(const PvIxParams *__restrict__ Xp)
{
    const PvIxParams X = *Xp;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= X.nseg || !X.cnt[s]) return;
    uint64_t p = X.start[s];
    uint64_t i = X.base[s];
    for (uint32_t k = 0; k < X.cnt[s] && i < X.max_records; k++, i++) {
        X.offs[i] = (uint32_t)p;
        p += 16 + (uint64_t)caplen_at(X.recs, p);
    }
}

// ts_sec change points (record i whose ts_sec differs from record i - 1's) and monotonicity,
// over n = min(records indexed, cap) records (n read on the device: no read-back between the
// scan and here). status: [1] change points, [2] out of order, [3] the last record's offset,
// [4] the last change point
extern "C" __global__ void pv_ix_secs(const PvIxParams *__restrict__ Xp, uint32_t cap)
{
    const PvIxParams X = *Xp;
    const uint32_t n = min(X.base[X.nseg], cap);
    auto sec_at = [&](uint64_t p) -> uint32_t {
        return ((p & 3) == 0) ? *reinterpret_cast<const uint32_t *>(X.recs + p)
                              : (uint32_t)X.recs[p] | ((uint32_t)X.recs[p + 1] << 8) | ((uint32_t)X.recs[p + 2] << 16) |
                                    ((uint32_t)X.recs[p + 3] << 24);
    };
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t p = X.offs[i];
        if (i == n - 1) X.status[3] = (uint32_t)p;
        const uint32_t sec = sec_at(p);
        const int64_t prev = i ? (int64_t)sec_at(X.offs[i - 1]) : -1;
        if ((int64_t)sec == prev) continue;
        if ((int64_t)sec < prev) atomicOr(&X.status[2], 1u);
        atomicMax(&X.status[4], i);
        const uint32_t k = atomicAdd(&X.status[1], 1u);
        if (k < X.max_changes) {
            X.sci[k] = i;
            X.scs[k] = sec;
        }
    }
}

// the offsets either side of the last change point (the ingest's cut at its last ts_sec
// boundary): status[5] = offs[last - 1], status[6] = offs[last]
extern "C" __global__ void pv_ix_cut(const PvIxParams *__restrict__ Xp)
{
    const PvIxParams X = *Xp;
    if (threadIdx.x != 0) return;
    const uint32_t k = X.status[4];
    if (k > 0) {
        X.status[5] = X.offs[k - 1];
        X.status[6] = X.offs[k];
    }
}
