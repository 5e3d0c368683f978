// SPDX-License-Identifier: MPL-2.0
//
// pv_ingest.cpp — host side of the pcap-record ingest.
//
// The reference walks a capture one record at a time on its input thread
// (PcapInputStream::_open_pcap, src/inputs/pcap/PcapInputStream.cpp:471-527). Here the
// host only has to produce the record offset index and the ts_sec change points of a
// block before it goes to the GPU, so that walk is split across host threads:
//
//   1. The block is cut into T byte segments. Thread 0 walks from the block start;
//      thread t > 0 guesses the first record start of its segment (the first offset
//      from which four consecutive headers are plausible: ts_sec near the block's first,
//      sub-second field in range, caplen <= min(len, 256 KiB)) and walks its segment
//      from there.
//   2. The guesses are then checked in segment order against the true chain: the true
//      first start of segment t is where segment t - 1's validated walk ended. Walks
//      are deterministic, so if that position is on thread t's list, the list from there
//      on IS the true chain; otherwise segment t is walked again from the true position.
//
// The result is bit-identical to the sequential walk (pv_index_records) for any input,
// plausible or not; the guesses only decide how much of the walk runs in parallel.
#include "pv_ingest.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace pvi {

Pool::Pool(unsigned nthreads)
{
    for (unsigned i = 1; i < std::max(1u, nthreads); i++) th_.emplace_back([this, i] { run(i); });
}

Pool::~Pool()
{
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
}

void Pool::run(unsigned)
{
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        while (next_ < n_) {
            const unsigned i = next_++;
            busy_++;
            lk.unlock();
            (*job_)(i);
            lk.lock();
            busy_--;
        }
        if (busy_ == 0) done_cv_.notify_all();
    }
}

void Pool::parallel_for(unsigned n, const std::function<void(unsigned)> &f)
{
    if (n == 0) return;
    if (th_.empty() || n == 1) {
        for (unsigned i = 0; i < n; i++) f(i);
        return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &f;
    n_ = n;
    next_ = 0;
    gen_++;
    cv_.notify_all();
    while (next_ < n_) {
        const unsigned i = next_++;
        busy_++;
        lk.unlock();
        f(i);
        lk.lock();
        busy_--;
    }
    done_cv_.wait(lk, [&] { return busy_ == 0 && next_ >= n_; });
    job_ = nullptr;
    n_ = 0;
}

unsigned default_threads()
{
    if (const char *e = getenv("PV_HOST_THREADS")) {
        const int v = atoi(e);
        if (v > 0) return (unsigned)std::min(v, 256);
    }
    const unsigned hc = std::thread::hardware_concurrency();
    return std::max(1u, std::min(hc ? hc : 1u, 16u));
}

void copy_parallel(Pool &pool, void *dst, const void *src, size_t bytes)
{
    const size_t piece = 4u << 20;
    const unsigned np = (unsigned)((bytes + piece - 1) / piece);
    pool.parallel_for(np, [&](unsigned i) {
        const size_t a = (size_t)i * piece, b = std::min(bytes, a + piece);
        memcpy((uint8_t *)dst + a, (const uint8_t *)src + a, b - a);
    });
}

namespace {

struct Hdr {
    uint32_t sec, frac, caplen, len;
};
inline Hdr hdr_at(const uint8_t *r, size_t pos)
{
    Hdr h;
    memcpy(&h, r + pos, 16);
    return h;
}

// One segment's walk: record starts in [lo, hi) from p, the position after the last
// record, and whether the walk stopped inside the segment (end of data / truncated record).
struct Seg {
    std::vector<uint64_t> pos;
    uint64_t end = 0;
    bool stopped = false;
    bool found = false;
};
void walk(const uint8_t *r, size_t bytes, uint64_t p, uint64_t hi, Seg &s)
{
    s.pos.clear();
    s.stopped = false;
    while (p < hi) {
        if (p + 16 > bytes) { s.stopped = true; break; }
        const uint32_t cl = hdr_at(r, p).caplen;
        if (p + 16 + (uint64_t)cl > bytes) { s.stopped = true; break; }
        s.pos.push_back(p);
        p += 16 + (uint64_t)cl;
    }
    s.end = p;
}
// ts_sec within a day of the block's first record, sub-second field in range, caplen at
// most 256 KiB and not above the original length: a 4-byte-shifted view of a capture
// whose caplen == len (ts_usec, caplen, len, next ts_sec) fails the ts_sec test
bool plausible(const uint8_t *r, size_t bytes, uint64_t p, uint32_t frac_lim, uint32_t sec0)
{
    for (int k = 0; k < 4; k++) {
        if (p == bytes) return true;
        if (p + 16 > bytes) return k > 0;
        const Hdr h = hdr_at(r, p);
        const uint32_t dsec = h.sec > sec0 ? h.sec - sec0 : sec0 - h.sec;
        if (dsec > 86400 || h.caplen > (256u << 10) || h.caplen > h.len || h.frac >= frac_lim) return false;
        if (p + 16 + (uint64_t)h.caplen > bytes) return k > 0;
        p += 16 + (uint64_t)h.caplen;
    }
    return true;
}

} // namespace

int index_records_parallel(Pool &pool, const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets,
                           uint64_t max_records, uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes,
                           pv_index_info *info, uint8_t *copy_dst)
{
    const unsigned T = pool.size();
    if (T <= 1 || bytes < (4u << 20) || bytes > 0xffffffffull) {
        if (copy_dst) copy_parallel(pool, copy_dst, recs, bytes);
        return pv_index_records(recs, bytes, ts_nano, offsets, max_records, sc_idx, sc_sec, max_changes, info);
    }
    const unsigned S = T * 2; // segments
    std::vector<uint64_t> lo(S + 1);
    for (unsigned t = 0; t <= S; t++) lo[t] = (uint64_t)bytes * t / S;
    std::vector<Seg> seg(S);
    const uint32_t frac_lim = ts_nano ? 1000000000u : 1000000u;
    const uint32_t sec0 = hdr_at(recs, 0).sec;
    // 1. guessed walks
    pool.parallel_for(S, [&](unsigned t) {
        // the segment's copy first (pinned staging): the walk then reads cache-warm bytes
        if (copy_dst) memcpy(copy_dst + lo[t], recs + lo[t], lo[t + 1] - lo[t]);
        uint64_t p = lo[t];
        if (t > 0) {
            const uint64_t lim = std::min<uint64_t>(lo[t + 1], lo[t] + (256u << 10) + 16);
            while (p < lim && !plausible(recs, bytes, p, frac_lim, sec0)) p++;
            if (p >= lim) return;
        }
        seg[t].found = true;
        seg[t].pos.reserve((lo[t + 1] - lo[t]) / 64 + 16);
        walk(recs, bytes, p, lo[t + 1], seg[t]);
    });
    // 2. validation along the true chain
    std::vector<uint64_t> first(S, 0), count(S, 0);
    uint64_t cur = 0;
    bool stopped = false;
    for (unsigned t = 0; t < S && !stopped; t++) {
        if (cur >= lo[t + 1]) continue; // no record starts inside this segment
        Seg &s = seg[t];
        auto it = s.found ? std::lower_bound(s.pos.begin(), s.pos.end(), cur) : s.pos.end();
        if (it != s.pos.end() && *it == cur) {
            first[t] = (uint64_t)(it - s.pos.begin());
        } else {
            walk(recs, bytes, cur, lo[t + 1], s);
            first[t] = 0;
        }
        count[t] = s.pos.size() - first[t];
        cur = s.end;
        stopped = s.stopped;
    }
    // 3. offsets (capped at max_records), in parallel
    std::vector<uint64_t> base(S + 1, 0);
    for (unsigned t = 0; t < S; t++) base[t + 1] = base[t] + count[t];
    const uint64_t total = base[S];
    const uint64_t n = std::min<uint64_t>(total, max_records);
    uint64_t used = cur;
    pool.parallel_for(S, [&](unsigned t) {
        for (uint64_t k = 0; k < count[t]; k++) {
            const uint64_t i = base[t] + k;
            if (i >= n) break;
            offsets[i] = (uint32_t)seg[t].pos[first[t] + k];
        }
    });
    if (n < total) used = offsets[n - 1] + 16 + (uint64_t)hdr_at(recs, offsets[n - 1]).caplen;
    // 4. ts_sec change points and monotonicity, in parallel over record ranges
    memset(info, 0, sizeof *info);
    info->monotone = 1;
    info->n_records = n;
    info->bytes_used = used;
    if (n == 0) return 0;
    const unsigned R = std::min<uint64_t>(S, (n + 4095) / 4096);
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> ch(R);
    std::vector<int> mono(R, 1);
    pool.parallel_for(R, [&](unsigned r) {
        const uint64_t a = n * r / R, b = n * (r + 1) / R;
        int64_t prev = a == 0 ? -1 : (int64_t)hdr_at(recs, offsets[a - 1]).sec;
        for (uint64_t i = a; i < b; i++) {
            const int64_t sec = hdr_at(recs, offsets[i]).sec;
            if (sec != prev) {
                if (sec < prev) mono[r] = 0;
                ch[r].emplace_back((uint32_t)i, (uint32_t)sec);
                prev = sec;
            }
        }
    });
    uint32_t nc = 0;
    for (unsigned r = 0; r < R; r++) {
        if (!mono[r]) info->monotone = 0;
        for (auto &e : ch[r]) {
            if (nc < max_changes) { sc_idx[nc] = e.first; sc_sec[nc] = e.second; }
            nc++;
        }
    }
    const Hdr h0 = hdr_at(recs, offsets[0]), h1 = hdr_at(recs, offsets[n - 1]);
    info->first_sec = h0.sec;
    info->first_nsec = ts_nano ? h0.frac : (int64_t)h0.frac * 1000;
    info->last_sec = h1.sec;
    info->last_nsec = ts_nano ? h1.frac : (int64_t)h1.frac * 1000;
    info->n_sec_changes = nc;
    if (nc > max_changes) return PV_ECAPACITY;
    return 0;
}

} // namespace pvi
