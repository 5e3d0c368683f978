// SPDX-License-Identifier: MPL-2.0
//
// pv_host.h — private to the host runtime (pv_host.cpp, pv_xshard.cpp): the context of one Net v1
// + DNS v1 handler pair on one GPU (pv_ctx), its bucket slots and windows, the host-compiled name
// fingerprint (pv_parse.h), the kernel entry points the runtime launches.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <arpa/inet.h>
#include <linux/if_packet.h>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <unordered_map>
#include <queue>
#include <set>
#include <tuple>
#include <vector>

#include <chrono>
#include <condition_variable>
#include <memory>

#include "pv_dnstap.h"
#include "pv_pcapng.h"
#include <thread>

#include "../../include/pvgpu.h"
#include "pv_ingest.h"
#include "pv_layout.h"

// The kernel's name fingerprint (pv_parse.h NameStats + fp56), compiled for the host so
// pv_set_dns_filters can key "only_qname" names exactly as the DNS pass keys first-query names.
namespace pvname {
#define PV_FN inline
#define PV_CREF(T) const T &
inline uint32_t pv_clz64(uint64_t x) { return (uint32_t)__builtin_clzll(x); }
inline uint32_t pv_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh)); }
#include "pv_parse.h"
#include "pv_psl_data.h"

// The device form of the public suffix table (pv_psl_data.h, generated from the reference's
// ICANN_DOMAINS): PV_PSL_SLOTS open-addressed slots of {FNV-1a of the label, byte offset,
// length, first suffix | count << 16} (length 0 = empty), then {byte offset, length} per
// suffix, then the strings. psl_match (pv_kernels.hip) reads it.
static std::vector<uint32_t> psl_blob()
{
    std::vector<uint32_t> w(PV_PSL_SFX_WORD + 2 * PV_PSL_NSFX, 0);
    std::string str;
    const size_t base = w.size() * 4;
    auto put = [&](const char *x) { const size_t o = base + str.size(); str += x; return (uint32_t)o; };
    uint32_t first = 0;
    for (uint32_t t = 0; t < PV_PSL_NTLD; t++) {
        const char *k = pv_psl_tld[t];
        uint32_t h = 0x811C9DC5u;
        for (const char *x = k; *x; x++) h = (h ^ (uint8_t)*x) * 16777619u;
        uint32_t s = h & (PV_PSL_SLOTS - 1);
        while (w[s * 4 + 2]) s = (s + 1) & (PV_PSL_SLOTS - 1);
        w[s * 4] = h; w[s * 4 + 2] = (uint32_t)strlen(k); w[s * 4 + 1] = put(k);
        w[s * 4 + 3] = first | ((uint32_t)pv_psl_count[t] << 16);
        first += pv_psl_count[t];
    }
    for (uint32_t j = 0; j < PV_PSL_NSFX; j++) {
        w[PV_PSL_SFX_WORD + 2 * j + 1] = (uint32_t)strlen(pv_psl_sfx[j]);
        w[PV_PSL_SFX_WORD + 2 * j] = put(pv_psl_sfx[j]);
    }
    str.resize((str.size() + 3) & ~(size_t)3, '\0');
    const size_t n0 = w.size();
    w.resize(n0 + str.size() / 4);
    memcpy(w.data() + n0, str.data(), str.size());
    return w;
}
inline uint64_t name_ph(const char *s, size_t n) // polynomial hash of the lower-case string
{
    uint64_t ph = 0;
    for (size_t k = 0; k < n; k++) ph = ph_step(ph, lower((uint8_t)s[k]));
    return ph;
}
// bounds-checked byte access to records in host memory (pv_shard_cuts)
struct HostRecs {
    const uint8_t *p;
    size_t n;
    uint32_t u8(uint64_t o) const { return o < n ? p[o] : 0u; }
    uint32_t u32(uint64_t o) const
    {
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) v |= u8(o + k) << (8 * k);
        return v;
    }
};
// the TCP stage's flow key of a record that may carry a DNS-over-TCP segment (tcp_seg_of,
// pv_kernels.hip: TCP with a DNS port on either side); false for any other record
inline bool tcp_dns_flow(const HostRecs &R, const PvParams &P, uint64_t rec, uint32_t *key)
{
    Parsed o;
    parse_record(R, parse_cfg(P), P, rec, o);
    if (o.l4 != 6) return false;
    const uint32_t pw = R.u32(o.l4off);
    auto bs = [](uint32_t x) { return ((x & 0xff) << 8) | ((x >> 8) & 0xff); };
    const uint32_t sp = bs(pw & 0xffff), dp = bs(pw >> 16);
    auto dns = [](uint32_t x) { return x == 53 || x == 5353 || x == 5355 || x == 53000; };
    if (!dns(sp) && !dns(dp)) return false;
    *key = flowkey(R, o);
    return true;
}
inline uint64_t name_fp(const char *s, size_t n)
{
    NameStats st;
    st.init();
    for (size_t k = 0; k < n; k++) st.put((uint8_t)s[k]);
    return fp56(st.ph, st.n, 0);
}
#undef PV_FN
#undef PV_CREF
} // namespace pvname

extern "C" __global__ void pv_net_kernel(const PvParams *P);
extern "C" __global__ void pv_net_kernel_ns(const PvParams *P);
extern "C" __global__ void pv_net_kernel_reg(const PvParams *P);
extern "C" __global__ void pv_net_kernel_reg_tc(const PvParams *P);
extern "C" __global__ void pv_net_kernel_span(const PvParams *P);
extern "C" __global__ void pv_store_blob(PvBlob b, uint4 *dst, uint32_t n16);
extern "C" __global__ void pv_fill_store(PvFillList L, PvBlob b, uint4 *dst, uint32_t n16);
extern "C" __global__ void pv_net_slow_list(const PvParams *P);
extern "C" __global__ void pv_rec_sizes(const uint8_t *recs, const uint32_t *offs, const uint8_t *trecs, const uint32_t *toffs,
                                        const uint32_t *idx, uint32_t stride, uint32_t n, uint32_t *sizes);
extern "C" __global__ void pv_rec_gather(const uint8_t *recs, const uint32_t *offs, const uint8_t *trecs, const uint32_t *toffs,
                                         const uint32_t *idx, uint32_t stride, uint32_t n, const uint32_t *dst_off, uint8_t *out);
extern "C" __global__ void pv_dns_kernel(const PvParams *P);
extern "C" __global__ void pv_dns_kernel_sfx(const PvParams *P);
extern "C" __global__ void pv_dns_kernel_f(const PvParams *P);
extern "C" __global__ void pv_dns_ecs(const PvParams *P);
extern "C" __global__ void pv_dns_suffix(const PvParams *P);
extern "C" __global__ void pv_fill_u64(uint64_t *p, uint64_t n, uint64_t v);
extern "C" __global__ void pv_fill_u32(uint32_t *p, uint64_t n, uint32_t v);
extern "C" __global__ void pv_fill_multi(PvFillList L);
extern "C" __global__ void pv_xact_compact(const PvParams *P, uint32_t b0, uint32_t kbase);
extern "C" __global__ void pv_dns_prescan(const PvParams *P);
extern "C" __global__ void pv_topn_combine(const PvParams *P);
extern "C" __global__ void pv_topn_combine_r12(const PvParams *P);
extern "C" __global__ void pv_topn_merge(const PvParams *P);
extern "C" __global__ void pv_topn_names_sfx(const PvParams *P);
extern "C" __global__ void pv_topn_name_fix(const PvParams *P, uint32_t tb);
extern "C" uint32_t pv_topn_merge_threads();
struct PvBpfIns;
extern "C" __global__ void pv_bpf_keep(const uint8_t *recs, const uint32_t *offs, uint32_t n, const PvBpfIns *prog, uint32_t ninsn,
                                       uint32_t *sz, uint32_t *kf);
extern "C" __global__ void pv_bpf_gather(const uint8_t *recs, const uint32_t *offs, uint32_t n, const uint32_t *sz, const uint32_t *boff,
                                         const uint32_t *rank, uint8_t *out, uint32_t *ooffs);
extern "C" __global__ void pv_bpf_secs(const uint8_t *out, const uint32_t *ooffs, uint32_t nk, uint32_t *flag, uint32_t *sec, uint32_t *down);
extern "C" __global__ void pv_bpf_secs_compact(const uint32_t *flag, const uint32_t *pos, const uint32_t *sec, uint32_t nk, uint32_t cap,
                                               uint32_t *sci, uint32_t *scs);
extern "C" hipError_t pv_exclusive_scan_u32(void *tmp, size_t *tmp_bytes, const uint32_t *in, uint32_t *out, size_t n, hipStream_t s);
extern "C" __global__ void pv_topn_xcount(const PvParams *P, PvXTabs T, uint32_t *cnt);
extern "C" __global__ void pv_topn_xscan(uint32_t reg_log2, uint32_t W, const uint32_t *cnt, uint32_t *off, uint32_t *hdr);
extern "C" __global__ void pv_topn_xwrite(const PvParams *P, PvXTabs T, const uint32_t *off, ulonglong2 *out);
extern "C" __global__ void pv_topn_xruns(uint32_t reg_log2, uint32_t W, uint32_t me, const uint32_t *hdr, uint32_t hdr_stride,
                                         uint64_t *cb_run);
extern "C" __global__ void pv_topn_xlookup(const PvParams *P, const uint64_t *keys, const uint32_t *tbs, uint32_t n, uint32_t *aux);
extern "C" __global__ void pv_net2_kernel(const PvParams *P);
extern "C" __global__ void pv_ix_guess(const PvIxParams *X);
extern "C" __global__ void pv_xv_hist(const PvXValue *v, const uint32_t *n_vals, uint32_t cap, uint32_t sg, uint32_t shift, PvXvSel sel,
                                      uint32_t *hist);
extern "C" __global__ void pv_ix_fix(const PvIxParams *X, uint32_t src);
extern "C" __global__ void pv_ix_scan(const PvIxParams *X);
extern "C" __global__ void pv_ix_write(const PvIxParams *X);
extern "C" __global__ void pv_ix_secs(const PvIxParams *X, uint32_t cap);
extern "C" __global__ void pv_ix_cut(const PvIxParams *X);
extern "C" __global__ void pv_topn_retry(const PvParams *P, const PvOvf *src, uint32_t n);
extern "C" __global__ void pv_xname_len(const uint8_t *arena, uint64_t arena_cap, const uint32_t *tb, const uint32_t *aux, uint32_t n,
                                        uint32_t *len);
extern "C" __global__ void pv_xname_copy(const uint8_t *arena, uint64_t arena_cap, const uint32_t *tb, const uint32_t *aux,
                                         const uint32_t *len, const uint64_t *off, uint32_t n, uint8_t *out);
extern "C" __global__ void pv_dns_tcp_filter(const PvParams *P);
extern "C" __global__ void pv_topn_purge(const PvParams *P, uint32_t tb, uint32_t *theta_out);
extern "C" __global__ void pv_topn_compact(const PvParams *P, uint32_t tb, uint8_t *tmp, unsigned long long *tmp_top);
extern "C" __global__ void pv_topn_names(const PvParams *P);
extern "C" __global__ void pv_xact_resolve(const PvXactParams *X);
extern "C" __global__ void pv_xact_resolve2(const PvXactParams *X);
extern "C" __global__ void pv_xact_slow_dev(const PvXactParams *X);
extern "C" __global__ void pv_xact_slow(const PvXactParams *X, uint32_t n_valid);
extern "C" __global__ void pv_xact_carry(const PvXactParams *X);
extern "C" __global__ void pv_xact_edge2(const PvXactParams *X, const PvEdgePair *pairs, uint32_t n, uint8_t *sfx, uint8_t *tsfx);
extern "C" __global__ void pv_xact_defer(const uint64_t *skeys, const uint32_t *svals, const PvXEvent *events, uint32_t n,
                                         PvXEvent *pend, uint64_t *pkeys, uint32_t *pvals, uint32_t at, uint32_t ehi,
                                         const uint64_t *eecs, uint64_t *pecs, uint32_t *ctr);
extern "C" __global__ void pv_xact_pend_in(uint64_t *skeys, uint32_t *svals, const uint64_t *pkeys, const uint32_t *pvals,
                                           uint32_t n_pend, uint32_t at);
extern "C" hipError_t pv_radix_sort_pairs(void *tmp, size_t *tmp_bytes, uint64_t *kin, uint64_t *kout, uint32_t *vin,
                                          uint32_t *vout, size_t n, hipStream_t s);
extern "C" __global__ void pv_dns_tcp(const PvParams *P);
extern "C" __global__ void pv_dnstap_kernel(const PvParams *P);
extern "C" __global__ void pv_tcp_keys(const PvTcpSeg *seg, uint32_t n, uint64_t *key, uint32_t *val);
extern "C" __global__ void pv_tcp_scan(const PvTcpParams *T);
extern "C" __global__ void pv_tcp_lookup(const PvTcpParams *T);
extern "C" __global__ void pv_tcp_insert(const PvTcpParams *T);
extern "C" __global__ void pv_tcp_flow(const PvTcpParams *T);
extern "C" __global__ void pv_tcp_migrate(const PvTcpParams *T);
extern "C" __global__ void pv_tcp_eoc(const PvTcpParams *T, const PvTcpSeg *seg, uint32_t n_seg, uint64_t *set, uint32_t set_mask,
                                      PvTcpSeg *out, uint32_t *cnt, uint32_t idx, uint32_t sec, uint32_t usec, uint32_t dir);
extern "C" hipError_t pv_tcp_sort(void *tmp, size_t *tmp_bytes, uint64_t *kin, uint64_t *kout, uint32_t *vin, uint32_t *vout,
                                  size_t n, hipStream_t s);

namespace pvh {

// status words (device): flags, n_events, n_resp, n_vals, DNS messages, new top-N names
enum { ST_FLAGS = 0, ST_NEV = 1, ST_NRESP = 2, ST_NVALS = 3, ST_NDNS = 4, ST_NNEW = 5, ST_TSEG = 6, ST_TSEG_BYTES = 7,
       ST_HANDS = 8 /* top-N handlers with entries (device only) */, ST_NKEYS = 9 /* key-list length */,
       ST_NSLOW = 10 /* general-path records the Net pass deferred (device only) */,
       ST_NECS = 11 /* top_ecs updates the DNS pass listed (device only) */, ST_WORDS = 12 };
// status allocation (zeroed per batch): the words above, padded
#define PV_NET_THREADS 256    // pv_net_kernel: four waves
#define PV_TRASH_WAVES 16384 // Net-pass waves with a 2-KiB trash area (grid <= 4096)
#define ST_ALLOC 32
#define PV_RESOLVE_PAD (30u << 10) // dynamic LDS of a v1 resolve workgroup: three workgroups a CU
#define ST_RB_WORDS (ST_ALLOC + PV_TABLES + 2) // status | tables' live counts | overflow words

struct SlotMeta {
    int64_t start_sec = 0, start_nsec = 0, end_sec = 0, end_nsec = 0;
    bool read_only = false;
    uint64_t period_length = 0;
    int64_t rel_base = 0;
    void set_read_only(int64_t s, int64_t ns)
    {
        end_sec = s; end_nsec = ns;
        period_length = (uint64_t)(end_sec - start_sec);
        read_only = true;
    }
};

// One handler's window (AbstractMetricsManager::_metric_buckets + _next_shift_tstamp,
// src/AbstractMetricsManager.h:233,264-305). The bucket of period ordinal k lives in slot
// k % PV_SLOTS of this handler's part of the device state.
enum { PART_NET = 0, PART_DNS = 1 };

// jsf32 (3rd/rng/jsf.h:38-70,111,151: jsf<uint32_t, uint32_t, 27, 17, 0>), the managers' deep
// sampling generator, default seed itype(0xcafe5eed00000001) = 1, 20 warm-up rounds
struct Jsf32 {
    uint32_t a = 0xf1ea5eedu, b = 1, c = 1, d = 1;
    Jsf32() { for (int i = 0; i < 20; i++) next(); }
    static uint32_t rot(uint32_t x, uint32_t k) { return (x << k) | (x >> (32 - k)); }
    uint32_t next()
    {
        const uint32_t e = a - rot(b, 27);
        a = b ^ rot(c, 17);
        b = c + d;
        c = d + e;
        d = e + a;
        return d;
    }
};
// One manager's deep-sampling draws, generated ahead by a producer thread: the draw sequence
// depends on nothing but the seed and the rate, so the bits (1 = deep: jsf32() % 100 < rate,
// AbstractMetricsManager::new_event :318-323) are ready before a batch needs them and the
// batch's serial work is a bit copy (Net: one draw per record) or a bit read per event (DNS).
class DrawStream {
  public:
    ~DrawStream() { stop(); }
    // the generator state the next start() draws from (a fresh Jsf32, or one stepped past a
    // shard's earlier draws)
    void reset(const Jsf32 &from)
    {
        stop();
        seed_ = from;
    }
    // the next draw (starting the producer at `rate` on first use)
    bool next(uint32_t rate)
    {
        if (!th_.joinable()) start(rate);
        if (tail_ == avail_) wait_more();
        const uint64_t k = tail_++;
        return (bits_[(k / 64) % kWords] >> (k % 64)) & 1;
    }
    // n draws as not-deep bits: bit i of out (32-bit words, zeroed by the caller) set when
    // draw i is not deep
    void take_not_deep(uint32_t rate, uint32_t *out, uint64_t n)
    {
        if (!th_.joinable()) start(rate);
        for (uint64_t i = 0; i < n;) {
            if (tail_ == avail_) wait_more();
            const uint64_t k = tail_, o = k % 64;
            const uint64_t m = std::min<uint64_t>({64 - o, n - i, avail_ - tail_});
            uint64_t v = ~(bits_[(k / 64) % kWords] >> o);
            if (m < 64) v &= (1ull << m) - 1;
            for (uint64_t b = 0; b < m;) {
                const uint64_t oi = i + b, ob = oi % 32, take = std::min<uint64_t>(32 - ob, m - b);
                out[oi / 32] |= (uint32_t)(((v >> b) & ((1ull << take) - 1)) << ob);
                b += take;
            }
            tail_ += m;
            i += m;
        }
    }

  private:
    static constexpr uint64_t kWords = 1u << 19; // at most 32M draws ahead
    static constexpr uint64_t kChunk = 1024;     // words the producer writes per round
    void start(uint32_t rate)
    {
        rng_ = seed_;
        rate_ = rate;
        bits_.assign(kWords, 0);
        head_ = tail_ = avail_ = done_ = 0;
        quit_ = false;
        th_ = std::thread([this] { produce(); });
    }
    void stop()
    {
        if (!th_.joinable()) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // publish what was consumed (the producer may reuse those words) and wait for more draws
    void wait_more()
    {
        std::unique_lock<std::mutex> g(mu_);
        done_ = tail_;
        cv_.notify_all();
        cv_.wait(g, [&] { return head_ > tail_; });
        avail_ = head_;
    }
    void produce()
    {
        for (;;) {
            uint64_t h;
            {
                std::unique_lock<std::mutex> g(mu_);
                // never overwrite the word holding the consumer's next draw
                cv_.wait(g, [&] { return quit_ || head_ / 64 + kChunk <= done_ / 64 + kWords; });
                if (quit_) return;
                h = head_ / 64;
            }
            for (uint64_t j = 0; j < kChunk; j++) {
                uint64_t v = 0;
                for (int b = 0; b < 64; b++) v |= (uint64_t)(rng_.next() % 100u < rate_) << b;
                bits_[(h + j) % kWords] = v;
            }
            {
                std::lock_guard<std::mutex> g(mu_);
                head_ = (h + kChunk) * 64;
            }
            cv_.notify_all();
        }
    }
    Jsf32 seed_, rng_;
    uint32_t rate_ = 100;
    std::vector<uint64_t> bits_;
    uint64_t head_ = 0, tail_ = 0, avail_ = 0, done_ = 0; // draw counts: produced, consumed, visible, released
    bool quit_ = false;
    std::mutex mu_;
    std::condition_variable cv_;
    std::thread th_;
};

struct Window {
    std::deque<uint32_t> slots; // front = live bucket
    int64_t next_shift_sec = 0;
    uint64_t ordinal = 0;       // period ordinal of the live bucket
    SlotMeta meta[PV_SLOTS];
    bool clean[PV_SLOTS] = {};  // slot part cleared and not written since
    uint32_t slot_at(uint64_t k) const { return (uint32_t)((ordinal + k) % PV_SLOTS); }
};

// ICON polynomial for lg_k = 11 (3rd/datasketches/cpc/include/icon_estimator.hpp:98-102)
const double ICON11[20] = {
    0.9999186020796150265, 0.3333249054574359826, 0.126791713589799987, -0.06662487271699729652,
    -0.07335552427910230211, 0.3316370184815959909, -1.434143797561290068, 4.180260309967409604,
    -8.593906870708760692, 12.95088874800289958, -14.56876092520539956, 12.37074367531410068,
    -7.969152075707960137, 3.888774396648960074, -1.424923326506990051, 0.385084561785229984,
    -0.07435541911616409816, 0.009695363567476529554, -0.0007644375960047160388, 2.75156194717188011e-05};

inline double icon11(uint32_t c)
{
    if (c < 2) return c == 0 ? 0.0 : 1.0;
    const double k = 2048.0, dc = (double)c;
    if (dc > 5.7 * k) return 0.7940236163830469 * k * pow(2.0, dc / k);
    const double x = dc / (2.0 * k);
    double t = ICON11[19];
    for (int j = 18; j >= 0; j--) t = t * x + ICON11[j];
    const double r = dc / k;
    const double res = dc * t * (1.0 + r * r * r / 66.774757);
    return res >= dc ? res : dc;
}

// HIP estimate replayed from coupons in first-occurrence order, with the
// sparse->windowed promotion and the kxp refresh of every 8th window move
// (cpc_sketch_impl.hpp:196-380).
inline double cpc_hip(std::vector<std::pair<int64_t, uint32_t>> &firsts)
{
    std::sort(firsts.begin(), firsts.end());
    std::vector<uint64_t> rows(2048, 0);
    static double kxp_byte[256];
    static bool init = false;
    if (!init) {
        for (int b = 0; b < 256; b++) {
            double s = 0;
            for (int c = 0; c < 8; c++) if (!((b >> c) & 1)) s += ldexp(1.0, -(c + 1));
            kxp_byte[b] = s;
        }
        init = true;
    }
    double kxp = 2048.0, hip = 0;
    uint32_t C = 0;
    int w = 0;
    bool windowed = false;
    for (auto &f : firsts) {
        uint32_t row = f.second >> 6, col = f.second & 63;
        rows[row] |= 1ull << col;
        C++;
        hip += 2048.0 / kxp;
        kxp -= ldexp(1.0, -(int)(col + 1));
        if (!windowed) {
            if (((uint64_t)C << 5) >= 3ull * 2048) windowed = true;
        } else if (((uint64_t)C << 3) >= (27ull + ((uint64_t)w << 3)) * 2048) {
            w++;
            if ((w & 7) == 0) {
                double bs[8] = {0};
                for (int i = 0; i < 2048; i++) {
                    uint64_t word = rows[i];
                    for (int j = 0; j < 8; j++) { bs[j] += kxp_byte[word & 0xff]; word >>= 8; }
                }
                double tot = 0;
                for (int j = 7; j >= 0; j--) tot += ldexp(1.0, -8 * j) * bs[j];
                kxp = tot;
            }
        }
    }
    return hip;
}

// libs/visor_dns/dns.h:31-265 name tables (IANA registry values, reference spellings)
inline const std::map<uint16_t, const char *> &qtype_names()
{
    static const std::map<uint16_t, const char *> m = {
        {0, "Reserved (0)"}, {1, "A"}, {2, "NS"}, {3, "MD"}, {4, "MF"}, {5, "CNAME"}, {6, "SOA"}, {7, "MB"},
        {8, "MG"}, {9, "MR"}, {10, "NULL"}, {11, "WKS"}, {12, "PTR"}, {13, "HINFO"}, {14, "MINFO"}, {15, "MX"},
        {16, "TXT"}, {17, "RP"}, {18, "AFSDB"}, {19, "X25"}, {20, "ISDN"}, {21, "RT"}, {22, "NSAP"},
        {23, "NSAP-PTR"}, {24, "SIG"}, {25, "KEY"}, {26, "PX"}, {27, "GPOS"}, {28, "AAAA"}, {29, "LOC"},
        {30, "NXT"}, {31, "EID"}, {32, "NIMLOC"}, {33, "SRV"}, {34, "ATMA"}, {35, "NAPTR"}, {36, "KX"},
        {37, "CERT"}, {38, "A6"}, {39, "DNAME"}, {40, "SINK"}, {41, "OPT"}, {42, "APL"}, {43, "DS"},
        {44, "SSHFP"}, {45, "IPSECKEY"}, {46, "RRSIG"}, {47, "NSEC"}, {48, "DNSKEY"}, {49, "DHCID"},
        {50, "NSEC3"}, {51, "NSEC3PARAM"}, {52, "TLSA"}, {53, "SMIMEA"}, {55, "HIP"}, {56, "NINFO"},
        {57, "RKEY"}, {58, "TALINK"}, {59, "CDS"}, {60, "CDNSKEY"}, {61, "OPENPGPKEY"}, {62, "CSYNC"},
        {63, "ZONEMD"}, {64, "SVCB"}, {65, "HTTPS"}, {99, "SPF"}, {100, "UINFO"}, {101, "UID"}, {102, "GID"},
        {103, "UNSPEC"}, {104, "NID"}, {105, "L32"}, {106, "L64"}, {107, "LP"}, {108, "EUI48"}, {109, "EUI64"},
        {249, "TKEY"}, {250, "TSIG"}, {251, "IXFR"}, {252, "AXFR"}, {253, "MAILB"}, {254, "MAILA"}, {255, "*"},
        {256, "URI"}, {257, "CAA"}, {258, "AVC"}, {259, "DOA"}, {260, "AMTRELAY"}, {32768, "TA"}, {32769, "DLV"},
        {65535, "Reserved (65535)"}};
    return m;
}
inline const std::map<uint16_t, const char *> &rcode_names()
{
    static const std::map<uint16_t, const char *> m = {
        {0, "NOERROR"}, {1, "FORMERR"}, {2, "SRVFAIL"}, {3, "NXDOMAIN"}, {4, "NOTIMP"}, {5, "REFUSED"},
        {6, "YXDOMAIN"}, {7, "YXRRSET"}, {8, "NXRRSET"}, {9, "NOTAUTH"}, {10, "NOTZONE"}, {11, "DSOTYPENI"},
        {16, "BADVERS"}, {17, "BADKEY"}, {18, "BADTIME"}, {19, "BADMODE"}, {20, "BADNAME"}, {21, "BADALG"},
        {22, "BADTRUNC"}, {23, "BADCOOKIE"}};
    return m;
}

// ---------------------------------------------------------------- JSON writer
struct Json {
    std::string s;
    std::vector<int> n{0};
    bool after_key = false;
    void sep()
    {
        if (after_key) { after_key = false; return; }
        if (n.back()++) s += ',';
    }
    void esc(const std::string &v)
    {
        s += '"';
        for (unsigned char c : v) {
            if (c == '"') s += "\\\"";
            else if (c == '\\') s += "\\\\";
            else if (c < 0x20 || c >= 0x80) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); s += b; } // bytes >= 0x80 as U+0080..U+00FF
            else s += (char)c;
        }
        s += '"';
    }
    Json &key(const std::string &k) { sep(); esc(k); s += ':'; after_key = true; return *this; }
    void str(const std::string &v) { sep(); esc(v); }
    void u(uint64_t v) { sep(); s += std::to_string(v); }
    void i(int64_t v) { sep(); s += std::to_string(v); }
    void d(double v)
    {
        sep();
        char b[40];
        snprintf(b, sizeof b, "%.17g", v);
        s += b;
        if (!strpbrk(b, ".eEn")) s += ".0";
    }
    void obj() { sep(); s += '{'; n.push_back(0); }
    void end_obj() { s += '}'; n.pop_back(); }
    void arr() { sep(); s += '['; n.push_back(0); }
    void end_arr() { s += ']'; n.pop_back(); }
};

inline bool hip_ok(hipError_t e) { return e == hipSuccess; }

} // namespace pvh
using namespace pvh;

// ---------------------------------------------------------------- context
// a value group's summary over every shard (pv_values_x_select)
struct XQuant {
    uint64_t n = 0, max = 0;
    std::vector<uint64_t> q;   // p50 p90 p95 p99 (value bits)
    std::vector<uint64_t> cdf; // counts at or below each hist_points() point (time kinds)
};

struct pv_ctx {
    std::vector<pv_bpf_insn> bpf; // the pcap input's BPF program (pv_set_bpf), empty = none
    // the program on the device and the filtered batch (pv_process_device runs the filter there)
    pv_bpf_insn *d_bpf = nullptr;
    size_t d_bpf_n = 0;
    bool bpf_dirty = false;
    uint32_t *d_fwork = nullptr; // 4 x max_records u32: sizes, keep flags, byte offsets, ranks
    uint8_t *d_frecs = nullptr;  // the kept records (max_records' bytes + PV_RECS_PAD)
    uint32_t *d_foffs = nullptr, *d_fsc = nullptr; // their offsets; change points (idx, sec) + counters
    void *d_fscan = nullptr;
    size_t fwork_n = 0, frecs_bytes = 0, fscan_bytes = 0;
    pv_config cfg{};
    std::string err;
    std::mutex mu;
    int device = 0;
    hipStream_t stream = nullptr;
    PvSubnets nets{};
    uint32_t ttl_s = 0, ttl_ms = 0;
    uint32_t net_groups = PV_NET_DEFAULT_GROUPS, dns_groups = PV_DNS_DEFAULT_GROUPS;
    uint32_t net2_groups = 0; // Net v2 attached: PV_NET2_* bits | PV_N2G_ON
    uint32_t dns2_groups = 0; // DNS v2 in place of v1: PV_DNS2_* bits | PV_N2G_ON
    float p90_2[3] = {0.0f, 0.0f, 0.0f}; // DNS v2 per-direction p90 of the last closed bucket (per_90th)
    // device state
    uint64_t *d_sum = nullptr;
    int64_t *d_cpc = nullptr;
    uint64_t *d_tkeys = nullptr, *d_tcnt = nullptr;
    uint32_t *d_taux = nullptr;
    uint8_t *d_arena = nullptr;
    uint64_t *d_arena_top = nullptr;
    uint64_t arena_cap = 128ull << 20; // per table; PV_ARENA_PARTS partitions
    uint32_t tcap_log2 = 22;
    PvXEvent *d_events = nullptr;
    uint64_t *d_ekeys = nullptr;
    uint32_t *d_blk_events = nullptr;
    uint64_t *d_mq = nullptr; // per-workgroup top-N update logs (grown on demand)
    uint64_t *d_tpbuf = nullptr; // the logs bucketed by table region (same size)
    uint64_t *d_cb = nullptr;    // combined update lists (same size)
    uint32_t *d_cb_cnt = nullptr;
    uint32_t *d_cb_h = nullptr;  // per combine workgroup: entries per region
    uint32_t cb_h_grid = 0;
    PvNewName *d_nn = nullptr;   // entries created by pv_topn_merge (names pending)
    uint64_t *d_iplog = nullptr; // dense IP log, one u64 per record (max_records + one tile)
    uint32_t *d_iplog32 = nullptr, *d_ipx_cnt = nullptr, *d_ipx_rep = nullptr; // compact IP log (register pass)
    uint64_t *d_ipdir = nullptr;
    uint32_t *d_slow = nullptr; // span Net pass: deferred record indices (max_records), their count
    uint64_t slow_cap = 0;
    uint4 *d_ecs = nullptr; // top_ecs updates of the UDP DNS pass (one per record at most)
    uint64_t ecs_cap = 0;
    uint64_t *d_trash = nullptr; // 64 B per Net-pass wave
    uint32_t nn_cap = 0;
    uint32_t reg_log2 = 0;
    size_t mq_bytes = 0;
    uint32_t *d_mq_cnt = nullptr;
    uint64_t *d_stamps = nullptr; // diagnostic phase stamps (PV_STAMPS env + -DPV_STAMPS build)
    int cus = 256;
    int wg_per_cu = 3;     // grid workgroups per CU (the batch's partition)
    bool wg_forced = false; // PV_NET_WGCU set: no per-batch choice
    bool dns_heavy = false; // the last batch was mostly DNS messages: four ranges per CU
    int reg_wg_per_cu = 1; // workgroups per CU of the register-window Net pass
    uint32_t cb_fan = 1;   // grid ranges per top-N combine workgroup
    int dns_wg_per_cu = 1; // resident workgroups per CU of the DNS pass (its register count)
    const char *net_kernel = "none"; // the Net-pass kernel the last span launched (pv_net_kernel_name)
    uint64_t *d_dq = nullptr; // DNS work lists (32-B messages)
    uint32_t *d_dq_cnt = nullptr;
    uint64_t *d_skeys = nullptr, *d_skeys2 = nullptr;
    uint32_t *d_svals = nullptr, *d_svals2 = nullptr;
    void *d_sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    PvXValue *d_xvals = nullptr;
    uint64_t xv_cap = 0; // values d_xvals holds (2 x max_records, doubled while it fits PV_XV_BUDGET_MB)
    uint32_t *d_xvh = nullptr, *h_xvh = nullptr; // pv_xv_hist's histograms (device, pinned read-back)
    PvXValid *d_valid = nullptr;
    uint32_t *d_nvals = nullptr;  // [0] values appended since reset, [1] deferred slow candidates, [2] carried queries
    // DNS queries still open at the end of the last batch (double-buffered), in sort-key
    // rank order; ranks of later records count from pend_base
    PvXEvent *d_pend[2] = {nullptr, nullptr};
    // DNS v2 top_ecs: the ECS address of each query event, and of each carried query
    uint64_t *d_eecs = nullptr, *d_pecs[2] = {nullptr, nullptr};
    uint64_t *d_pkeys[2] = {nullptr, nullptr};
    uint32_t *d_pvals[2] = {nullptr, nullptr}; // each carried query's index in the event store d_pend
    uint32_t pend_cur = 0;
    uint64_t n_pend = 0, pend_cap = 0;
    // event store: capacity of d_events / d_pend (equal, so a query-only batch's store can be
    // handed over), extent of d_pend[pend_cur] in use; key list capacity (d_skeys / d_pkeys)
    uint64_t ev_store_cap = 0, pend_hi = 0, key_cap = 0;
    int64_t pend_base = -1;
    // shard-edge stubs (orphan responses) accumulated since reset, device counter in d_nvals[3]
    PvXEvent *d_orph = nullptr;
    uint32_t orph_cap = 0;
    std::vector<std::pair<int64_t, uint32_t>> dns_shifts; // (threshold second, new DNS slot) since reset
    uint32_t gen[PV_SLOTS] = {0}; // bumped when a DNS slot is recycled; values carry slot | gen << 8
    uint64_t *d_dbits = nullptr;  // pv_dns_prescan output (one bit per record)
    uint64_t *h_dbits = nullptr;  // pinned host copy
    size_t xvals_synced = 0;
    float from90 = 0.0f, to90 = 0.0f; // DnsMetricsManager::_from90th / _to90th
    uint32_t *d_status = nullptr;
    // bounded top-N tables: entries per table (device, read back with each batch's status),
    // each purged region's accumulated theta (the estimate offset of its survivors)
    uint32_t *d_tab_live = nullptr, *h_tab_live = nullptr, *d_theta = nullptr;
    PvOvf *d_ovf = nullptr, *d_ovf2 = nullptr; // top-N overflow list and its retry copy
    uint32_t *d_ovf_cnt = nullptr, ovf_cap = 0;
    uint32_t *h_ovf = nullptr;                  // pinned copy of the two overflow words (read with the status)
    bool ovf_known = false;                     // h_ovf read back after the transaction stage's resolve
    uint64_t ovf_rounds = 0;                    // purge-and-retry rounds so far
    uint8_t *d_ctmp = nullptr;          // arena compaction scratch (one table's arena)
    unsigned long long *d_ctop = nullptr;
    std::vector<uint64_t> roff[PV_TABLES];
    uint64_t purges = 0;
    // DNS v1 filters (pv_set_dns_filters): PVF_* bits, only_rcode mask, answer_count, only_qtype
    uint32_t f_flags = 0, f_rcode_mask = 0, f_ancount = 0, f_nq = 0;
    uint16_t f_qt[PV_MAX_QTYPES] = {};
    uint32_t f_nqn = 0;
    uint64_t f_qn[PV_MAX_QNAMES] = {};
    uint8_t *d_sfx = nullptr; // only_qname_suffix: suffix_size per record of the batch (names kernels)
    uint32_t *d_psl = nullptr; // public_suffix_list table (psl_blob)
    uint32_t f_nsx = 0, f_sxl[PV_MAX_SUFFIXES] = {};
    uint64_t f_sxh[PV_MAX_SUFFIXES] = {};
    PvParams *d_params = nullptr;      // kernel parameter blocks (device memory)
    // pinned host mirrors of the per-batch uploads and the status read-back (direct DMA,
    // no pageable staging copy on the stream)
    PvParams *h_params = nullptr;
    PvXactParams *h_xparams = nullptr;
    uint32_t *h_status = nullptr;
    PvXactParams *d_xparams = nullptr;
    uint64_t max_records = 0;
    // host-memory ingest (pv_process_host): worker pool, copy stream and two staging
    // slots (pinned host chunk + offsets, device chunk + offsets)
    struct Stage {
        uint8_t *h_recs = nullptr, *d_recs = nullptr;
        uint32_t *h_offs = nullptr, *d_offs = nullptr;
        hipEvent_t copied = nullptr;
        std::vector<uint32_t> sci, scs;
        pv_index_info info{};
        // device record index (pv_index.hip): segment state, status words, change points
        uint8_t *d_ix = nullptr;    // PvIxParams + arrays, one allocation
        PvIxParams *h_ix = nullptr; // pinned: params, then status / small read-backs
        uint32_t ix_nseg = 0;
        uint32_t cut_o[2] = {0, 0}; // offsets of the records either side of the last ts_sec change
        bool last = false;          // host-index ingest: the data's final batch
    };
    bool device_index = true; // PV_INGEST_INDEX=host selects the host walk
    // device-index ingest ring: raw chunks land at offset chunk of 2 x chunk buffers, the
    // previous chunk's tail (records after its ts_sec cut) is moved in front of them on the device
    struct Ring {
        uint8_t *d_buf = nullptr;
        uint32_t *d_offs = nullptr;
        uint8_t *h_stage = nullptr;         // pinned staging of a pageable source
        hipEvent_t landed = nullptr;
    } ring[8];
    uint32_t ring_n = 4; // slots in use (PV_INGEST_RING, 3..8): the producer runs ring_n - 2 pieces ahead
    hipStream_t copy_stream2 = nullptr;
    std::unique_ptr<pvi::Pool> pool;
    Stage stage[2];
    size_t stage_bytes = 0;   // record bytes per chunk
    uint64_t stage_recs = 0;  // records per chunk
    hipStream_t copy_stream = nullptr;
    double ingest_ms[4] = {0, 0, 0, 0}; // host copy, index, H2D issue, device processing (pv_ingest_timing)
    // PV_HOST_PROF: host wall time between marks of the ingest loop and the batch (HP), printed by pv_destroy
    bool hprof_on = getenv("PV_HOST_PROF") != nullptr;
    double hprof[20] = {};
    std::chrono::steady_clock::time_point hp_t = std::chrono::steady_clock::now();
    // window state: the Net and DNS managers shift independently
    Window net, dns;
    bool started = false, ended = false;
    int64_t last_sec = 0, last_nsec = 0;
    uint64_t global_base = 0, records_seen = 0;
    // host copies of transaction values, per slot/kind
    std::vector<PvXValue> xvals_host;
    // merged top-N records from other ranks: table -> key -> (count, name)
    std::map<uint32_t, std::map<uint64_t, std::pair<uint64_t, std::string>>> remote_topn;
    // multi-GPU top-N exchange (pv_topn_x_*, pv_comm_merge_topn): device scratch, and the merged
    // view: this rank's regions of x_ranks (0: not merged), then every owner's leading entries
    uint32_t *d_xcnt = nullptr, *d_xrhdr = nullptr;
    uint64_t *d_xtot = nullptr;
    void *d_xsend = nullptr, *d_xrecv = nullptr;
    size_t xcnt_bytes = 0, xrhdr_bytes = 0, xtot_bytes = 0, xsend_bytes = 0, xrecv_bytes = 0;
    PvParams *d_xp = nullptr;
    uint32_t x_ranks = 0, x_rank = 0;
    bool x_view_on = false;
    // a merge across ranks (bucket all-reduce, top-N owner exchange, shard edges, merged values)
    // rewrote this context's window with other shards' data: the merged window is terminal, and
    // batches are refused until pv_reset (merged_refuse)
    bool merged = false;
    const char *merged_by = nullptr;
    std::map<uint32_t, std::map<uint64_t, std::pair<uint64_t, std::string>>> x_view; // part << 16 | slot mask -> key -> (estimate, name)
    // merged quantile inputs (pv_values_x_select): per (DNS slot set as a bit mask, value kind)
    std::map<std::pair<uint32_t, uint32_t>, XQuant> xq;
    bool xq_on = false;
    // device fills not launched yet (launch_fill*; one pv_fill_multi per flush_fills)
    PvFillList fills{};
    uint64_t fills_max = 0;
    // kernel timing (pv_kernel_timing): the Net pass of every timing_every-th batch (0: none)
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    double kernel_ms = 0;
    uint64_t kernel_launches = 0;
    uint32_t timing_every = 0;
    uint64_t timing_ctr = 0;
    // RCCL communicator (pv_comm_*)
    ncclComm_t comm = nullptr;
    int comm_ranks = 0, comm_rank = 0;
    // DNS over TCP (pv_tcp.hip): segments emitted per batch, the TCP record tile masks and
    // their prefix maxima; the stage's buffers (allocated on first use), the flow table and
    // the double-buffered carry arena with its carried-flow lists
    PvTcpSeg *d_tseg = nullptr;
    uint32_t tseg_cap = 0;
    uint64_t *d_tmask = nullptr;
    uint32_t *d_tpm = nullptr;
    uint32_t *d_tcpcnt = nullptr, *h_tcpcnt = nullptr; // PVT_WORDS, then the LT carry word
    PvTcpParams *d_tparams = nullptr, *h_tparams = nullptr;
    bool tcp_alloced = false;
    uint64_t *d_tkey[2] = {nullptr, nullptr};
    uint32_t *d_tval[2] = {nullptr, nullptr};
    uint32_t *d_run_flow = nullptr;
    void *d_tsort_tmp = nullptr;
    size_t tsort_tmp_bytes = 0;
    PvTcpFlow *d_flows = nullptr;
    uint32_t flow_cap_log2 = 18;
    uint8_t *d_carry[2] = {nullptr, nullptr};
    uint64_t carry_cap[2] = {0, 0};
    uint32_t *d_clist[2] = {nullptr, nullptr};
    uint32_t carry_cur = 0, n_clist = 0;
    uint64_t carry_used = 0;
    PvTcpFrag *d_frags = nullptr;
    uint32_t frag_cap = 0;
    uint8_t *d_marena = nullptr;
    uint64_t marena_cap = 0;
    uint32_t *d_moffs = nullptr;
    uint64_t *d_tmq = nullptr; // 32-B DnsMsg items
    uint8_t *d_tsfx = nullptr;
    uint32_t tmsg_cap = 0;
    uint32_t tcp_stage = 0;   // stage ordinal (flow entries remember the last one that touched them)
    bool tcp_active = false;  // a stage has run since the last reset
    // the end of the capture (pv_set_end_of_capture): armed for the next processing call, which
    // marks its final batch (eoc_batch) and that batch's last TCP stage (eoc_stage); in_host: inside
    // pv_process_host, whose ingest loops mark the final batch themselves
    bool eoc_armed = false, eoc_batch = false, eoc_stage = false, in_host = false;
    PvTcpSeg *d_eoc = nullptr; // close segments of the open connections (eoc_cap: flow table + batch segments)
    uint64_t eoc_cap = 0;
    uint32_t *d_eoc_cnt = nullptr;
    bool tcp_pre = false;     // this batch's stage runs ahead of the Net pass (prescan emits)
    uint32_t tcp_nmsg = 0;    // messages of the current batch
    // tcp_packet_reassembly_cache_limit (0: not set). In the exact LRU mode PcapInputStream's LRU
    // list of connections is replayed on the host across batches (front = most recently put;
    // value = the put's second: ConnectionData's endTime, 0 before a connection's second packet)
    uint64_t tcp_limit = 0;
    // dnstap input proxy's only_hosts (DnstapInputEventProxy, src/inputs/dnstap/DnstapInputStream.h:96-146)
    bool dt_only_hosts = false;
    std::vector<std::pair<uint32_t, uint32_t>> dt_v4; // network (network order), cidr
    std::vector<std::pair<std::array<uint8_t, 16>, uint32_t>> dt_v6;
    std::list<std::pair<uint32_t, uint32_t>> lru;
    std::unordered_map<uint32_t, std::list<std::pair<uint32_t, uint32_t>>::iterator> lru_at;
    // connections whose close would deliver held fragments (PVT_EV_HOLD after their last segment)
    std::set<uint32_t> lru_hold;
    bool tcp_exact = false;   // pv_set_tcp_exact_lru
    bool tcp_exact_on() const { return tcp_exact || tcp_limit; }
    uint32_t *d_lru_ev = nullptr, *d_fclose = nullptr;
    uint64_t lru_ev_cap = 0, fclose_cap = 0;
    // deep sampling (deep_sample_rate < 100): each manager's generator, the span's "not deep"
    // bitmaps (Net by record, DNS by the record of its event), pinned staging + device copies
    uint32_t sample_rate = 100;
    DrawStream draws_net, draws_dns;
    bool dns_deep_now = true;   // the DNS manager's _deep_sampling_now (a filtered event counts it)
    uint64_t plan_draws = 0;    // DNS draws (unfiltered DNS events) pv_dns_event_seconds_host counted
    uint64_t *d_fbits = nullptr, *h_fbits = nullptr;   // per record: a filtered DNS event (sampling)
    uint64_t *d_tfbits = nullptr, *h_tfbits = nullptr; // per TCP message
    uint32_t *d_ntcp = nullptr, *h_ntcp = nullptr;     // per TCP message: not deep
    uint64_t tmsg_bits_cap = 0;                        // messages the three TCP bitmaps hold
    std::vector<std::pair<uint64_t, uint32_t>> tcp_items; // (ord, message item) of the batch, by ord
    uint32_t *h_ndeep = nullptr, *d_ndeep = nullptr;
    uint64_t ndeep_words = 0;
    std::vector<std::pair<uint64_t, int64_t>> tcp_ords; // (ord, second) of the batch's messages, by ord
    // sharded top_slow (pv_set_slow_defer): the DNS period ordinal of each slot | generation,
    // the deferred slow-transaction candidates with their response records, and the records of
    // the orphan stubs (in d_orph order), which may become edge pairs
    bool slow_defer = false;
    std::unordered_map<uint32_t, uint64_t> sg_ord;
    struct SlowCand {
        uint64_t ord, us;
        uint32_t off;      // record in sstore
        uint8_t dir, tcp;
    };
    std::vector<uint8_t> sstore;
    std::vector<SlowCand> scands, sorph;
    uint32_t orph_done = 0;
    size_t xv_local_end = SIZE_MAX;     // xvals_host entries of this rank's own batches
    std::vector<std::pair<uint64_t, PvXValue>> slow_xv; // edge-pair times by period ordinal
    // shard-edge stubs kept on the host (sharded runs): the first event of a key in this shard
    // that may meet a query an earlier shard leaves open (orphan responses, first queries below
    // the edge horizon), in stream order, with the record of a response (for top_slow)
    struct EdgeStub {
        PvXEvent e;
        uint64_t ord;
        int64_t cand;  // SlowCand template in sorph (responses), -1 for queries
        int64_t order; // DNS v2: first-occurrence order (the response's qname CPC order as an edge pair)
    };
    int64_t *d_orph_ord = nullptr; // DNS v2 stubs' orders (pv_set_slow_defer)
    std::vector<EdgeStub> stubs;
    int64_t edge_h = 0;                                        // first record second + ttl + 61
    std::vector<std::pair<int64_t, uint64_t>> dns_shift_ord;   // (threshold second, ordinal) of local DNS shifts

    int fail(int code, const char *fmt, ...)
    {
        char b[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(b, sizeof b, fmt, ap);
        va_end(ap);
        err = b;
        return code;
    }
    int hipfail(hipError_t e, const char *what)
    {
        return fail(PV_EHIP, "%s: %s", what, hipGetErrorString(e));
    }
};

// PV_HOST_PROF mark k: host time since the previous mark goes to hprof[k]
#define HP(k)                                                                                      \
    do {                                                                                           \
        if (c->hprof_on) {                                                                         \
            const auto n_ = std::chrono::steady_clock::now();                                      \
            c->hprof[k] += std::chrono::duration<double, std::milli>(n_ - c->hp_t).count();        \
            c->hp_t = n_;                                                                          \
        }                                                                                          \
    } while (0)


// ---- shared by pv_host.cpp, pv_render.cpp and pv_xshard.cpp
namespace pvh {
// device-side top-N records of one table: (key, count, name) (pv_render.cpp read_topn)
struct TopRec {
    uint64_t key;
    uint64_t count;
    std::string name;
};
int read_topn(pv_ctx *c, uint32_t s, std::vector<TopRec> &out); // s: table (PV_TSLOT)
// the bucket slots of a window period (merged: the first `period` slots)
int window_slots(pv_ctx *c, const Window &w, uint32_t period, bool merged, std::vector<uint32_t> &out);
void flush_fills(pv_ctx *c);
int launch_fill32(pv_ctx *c, uint32_t *p, uint64_t n, uint32_t v);
void clear_part(pv_ctx *c, int part, uint32_t s);
void win_shift(pv_ctx *c, Window &w, int64_t T, int64_t Tns = 0);
uint32_t host_metric(const pv_ctx *c, uint64_t key);
const std::vector<uint64_t> &hist_points();
uint64_t quantile_at(std::vector<uint64_t> v, double r);
int sync_xvals(pv_ctx *c);
// the merge entry points rewrite the window with other shards' data (note at pv_ctx::merged)
void mark_merged(pv_ctx *c, const char *by);
} // namespace pvh
extern "C" {
namespace pvh {
void params_common(pv_ctx *c, PvParams &P, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n);
int drain_overflow(pv_ctx *c, hipStream_t st, bool known = false, bool *drained = nullptr, const PvParams *dP = nullptr);
} // namespace pvh
}
