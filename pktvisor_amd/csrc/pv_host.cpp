// SPDX-License-Identifier: MPL-2.0
//
// pv_host.cpp — host runtime behind include/pvgpu.h.
//
// Owns the device state of one Net v1 + DNS v1 handler pair on one GPU:
// bucket slots (ring of PV_SLOTS), the window of the last num_periods buckets,
// period-shift bookkeeping (AbstractMetricsManager::new_event/_period_shift,
// src/AbstractMetricsManager.h:276-333), the transaction pairing pass, and the
// finalisation of device buckets into the reference's JSON shape
// (NetworkMetricsBucket::to_json net/v1 ...cpp:447-505, DnsMetricsBucket::to_json
// dns/v1 ...cpp:735-836, window_merged_json AbstractMetricsManager.h:601-647).
//
// Sketch outputs: counters and dense tables are exact; top-N estimates are
// exact counts (inside the FI sketch's stated error bound, which allows
// [true, true + 3.5/2^13 * N]); quantiles are exact under the KLL rank rule
// (identical to KLL while n <= 200, within its rank error beyond); CPC is the
// reference estimator replayed exactly from per-coupon first-occurrence indices
// (HIP for a single bucket, ICON after a union), bit-identical to datasketches.
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
extern "C" __global__ void pv_dns_suffix(const PvParams *P);
extern "C" __global__ void pv_fill_u64(uint64_t *p, uint64_t n, uint64_t v);
extern "C" __global__ void pv_fill_u32(uint32_t *p, uint64_t n, uint32_t v);
extern "C" __global__ void pv_fill_multi(PvFillList L);
extern "C" __global__ void pv_xact_compact(const PvParams *P, uint32_t b0, uint32_t kbase);
extern "C" __global__ void pv_dns_prescan(const PvParams *P);
extern "C" __global__ void pv_topn_combine(const PvParams *P);
extern "C" __global__ void pv_topn_combine_r12(const PvParams *P);
extern "C" __global__ void pv_topn_merge(const PvParams *P);
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

namespace {

// status words (device): flags, n_events, n_resp, n_vals, DNS messages, new top-N names
enum { ST_FLAGS = 0, ST_NEV = 1, ST_NRESP = 2, ST_NVALS = 3, ST_NDNS = 4, ST_NNEW = 5, ST_TSEG = 6, ST_TSEG_BYTES = 7,
       ST_HANDS = 8 /* top-N handlers with entries (device only) */, ST_NKEYS = 9 /* key-list length */,
       ST_NSLOW = 10 /* general-path records the Net pass deferred (device only) */, ST_WORDS = 11 };
// status allocation (zeroed per batch): the words above, padded
#define PV_NET_THREADS 256    // pv_net_kernel: four waves
#define PV_TRASH_WAVES 16384 // Net-pass waves with a 2-KiB trash area (grid <= 4096)
#define ST_ALLOC 32
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

double icon11(uint32_t c)
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
double cpc_hip(std::vector<std::pair<int64_t, uint32_t>> &firsts)
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
const std::map<uint16_t, const char *> &qtype_names()
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
const std::map<uint16_t, const char *> &rcode_names()
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

} // namespace

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

namespace {

int parse_host_spec(pv_ctx *c, const char *spec)
{
    if (!spec) return 0;
    std::string s = spec;
    size_t pos = 0;
    while (pos < s.size()) {
        size_t e = s.find(',', pos);
        std::string host = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
        pos = e == std::string::npos ? s.size() : e + 1;
        if (host.empty()) continue;
        // libs/visor_utils/utils.cpp:128-164 (same error strings)
        size_t d = host.find('/');
        if (d == std::string::npos) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        std::string ip = host.substr(0, d), cs = host.substr(d + 1);
        if (cs.empty() || !std::all_of(cs.begin(), cs.end(), ::isdigit)) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        int cidr = atoi(cs.c_str());
        if (ip.find(':') != std::string::npos) {
            if (cidr < 0 || cidr > 128) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (c->nets.n6 >= PV_MAX_SUBNETS) return c->fail(PV_EINVAL, "too many host subnets");
            uint8_t a[16];
            if (inet_pton(AF_INET6, ip.c_str(), a) != 1) return c->fail(PV_EINVAL, "invalid IPv6 address: %s", ip.c_str());
            memcpy(c->nets.v6_addr[c->nets.n6], a, 16);
            c->nets.v6_cidr[c->nets.n6++] = (uint32_t)cidr;
        } else {
            if (cidr < 0 || cidr > 32) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (c->nets.n4 >= PV_MAX_SUBNETS) return c->fail(PV_EINVAL, "too many host subnets");
            in_addr a;
            if (inet_pton(AF_INET, ip.c_str(), &a) != 1) return c->fail(PV_EINVAL, "invalid IPv4 address: %s", ip.c_str());
            uint32_t i = c->nets.n4++;
            c->nets.v4_addr[i] = a.s_addr;
            c->nets.v4_all[i] = cidr == 0;
            c->nets.v4_mask[i] = cidr == 0 ? 0 : htonl(0xFFFFFFFFu << (32 - cidr));
        }
    }
    return 0;
}

// Device fills are queued and launched together by flush_fills (one kernel instead of
// one per region); every path that launches kernels or reads device state flushes first.
void flush_fills(pv_ctx *c)
{
    if (!c->fills.n) return;
    hipSetDevice(c->device);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((c->fills_max + 255) / 256, 4096);
    hipLaunchKernelGGL(pv_fill_multi, dim3(blocks), dim3(256), 0, c->stream, c->fills);
    c->fills.n = 0;
    c->fills_max = 0;
}
void queue_fill(pv_ctx *c, void *p, uint64_t n, uint64_t v, uint32_t w32)
{
    if (!n) return;
    if (c->fills.n == PV_FILL_SEGS) flush_fills(c);
    c->fills.s[c->fills.n++] = PvFillSeg{p, n, v, w32, 0};
    c->fills_max = std::max(c->fills_max, n);
}
int launch_fill64(pv_ctx *c, uint64_t *p, uint64_t n, uint64_t v)
{
    queue_fill(c, p, n, v, 0);
    return 0;
}
int launch_fill32(pv_ctx *c, uint32_t *p, uint64_t n, uint32_t v)
{
    queue_fill(c, p, n, v, 1);
    return 0;
}

// Clear one handler's part of a slot on the device (enqueued on the context stream):
// its SUM and MIN words and its top-N table. A part that is still clean is skipped.
void clear_part(pv_ctx *c, int part, uint32_t s)
{
    Window &w = part == PART_NET ? c->net : c->dns;
    if (part == PART_DNS) {
        // quantile inputs of the slot's previous bucket no longer match (bounded host memory)
        c->gen[s] = (c->gen[s] + 1) & 0xffffff;
        // (a sharded run keeps them: the merge computes every period's slow thresholds)
        if (!c->slow_defer)
            c->xvals_host.erase(std::remove_if(c->xvals_host.begin(), c->xvals_host.end(),
                                               [s](const PvXValue &v) { return (v.slot & 0xff) == s; }),
                                c->xvals_host.end());
    }
    const uint32_t t = s + (part == PART_DNS ? PV_SLOTS : 0);
    c->remote_topn.erase(t);
    c->x_view.clear(); // (its slot sets name slots)
    w.meta[s] = SlotMeta();
    if (w.clean[s]) return;
    const uint64_t tcap = 1ull << c->tcap_log2;
    uint64_t *sum = c->d_sum + (uint64_t)s * PV_SUM_WORDS;
    uint64_t *cpc = (uint64_t *)c->d_cpc + (uint64_t)s * PV_MIN_WORDS;
    if (part == PART_NET) {
        launch_fill64(c, sum, PV_SUM_NET_WORDS, 0);
        launch_fill64(c, cpc, PV_MIN_NET_WORDS, (uint64_t)PV_CPC_EMPTY);
    } else {
        launch_fill64(c, sum + PV_OFF_DNS, PV_SUM_WORDS - PV_OFF_DNS, 0);
        launch_fill64(c, cpc + PV_MIN_NET_WORDS, PV_MIN_WORDS - PV_MIN_NET_WORDS, (uint64_t)PV_CPC_EMPTY);
    }
    // keys only: a count or name word is read only behind a non-zero key, and whoever
    // claims an entry overwrites its name word and adds net of the stale count (global_add,
    // pv_topn_merge)
    launch_fill64(c, c->d_tkeys + t * tcap, tcap, 0);
    launch_fill64(c, c->d_arena_top + (uint64_t)t * PV_ARENA_PARTS, PV_ARENA_PARTS, 0);
    launch_fill32(c, c->d_tab_live + t, 1, 0);
    c->roff[t].clear();
    w.clean[s] = true;
}

// _period_shift (src/AbstractMetricsManager.h:276-305) on the host mirror of one window: the
// live bucket becomes read-only at T, the next ordinal's slot (reserved and cleared before
// the batch that shifts) becomes live, the oldest beyond num_periods drops out.
void win_shift(pv_ctx *c, Window &w, int64_t T, int64_t Tns = 0)
{
    w.meta[w.slots.front()].set_read_only(T, Tns);
    w.ordinal++;
    const uint32_t s = w.slot_at(0);
    w.meta[s] = SlotMeta();
    w.meta[s].start_sec = T;
    w.meta[s].start_nsec = Tns;
    w.slots.push_front(s);
    if (w.slots.size() > c->cfg.num_periods) w.slots.pop_back();
    w.next_shift_sec = T + 60;
    if (&w == &c->dns) c->sg_ord[s | (c->gen[s] << 8)] = w.ordinal;
}

int ensure_started(pv_ctx *c, int64_t sec, int64_t nsec)
{
    if (c->started) return 0;
    // set_start_tstamp on both managers (AbstractMetricsManager.h:423-431)
    for (int part : {PART_NET, PART_DNS}) {
        Window &w = part == PART_NET ? c->net : c->dns;
        w.ordinal = 0;
        clear_part(c, part, 0);
        w.meta[0].start_sec = sec;
        w.meta[0].start_nsec = nsec;
        w.slots.assign(1, 0);
        w.next_shift_sec = sec + 60;
    }
    c->sg_ord[0 | (c->gen[0] << 8)] = 0;
    c->started = true;
    return 0;
}

// Device-side top-N records of one table: (key, count, name)
struct TopRec {
    uint64_t key;
    uint64_t count;
    std::string name;
};

int read_topn(pv_ctx *c, uint32_t s, std::vector<TopRec> &out) // s: table (PV_TSLOT)
{
    flush_fills(c);
    uint64_t tcap = 1ull << c->tcap_log2;
    std::vector<uint64_t> keys(tcap), cnt(tcap);
    std::vector<uint32_t> aux(tcap);
    uint64_t tops[PV_ARENA_PARTS];
    hipError_t e;
    if (!hip_ok(e = hipMemcpyAsync(keys.data(), c->d_tkeys + s * tcap, tcap * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(cnt.data(), c->d_tcnt + s * tcap, tcap * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(aux.data(), c->d_taux + s * tcap, tcap * 4, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(tops, c->d_arena_top + (uint64_t)s * PV_ARENA_PARTS, sizeof tops, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "read top-N table");
    const uint64_t pcap = c->arena_cap / PV_ARENA_PARTS;
    std::vector<std::vector<uint8_t>> parts(PV_ARENA_PARTS);
    for (uint32_t p = 0; p < PV_ARENA_PARTS; p++) {
        uint64_t used = std::min<uint64_t>(tops[p], pcap);
        parts[p].resize(used);
        if (used && !hip_ok(e = hipMemcpy(parts[p].data(), c->d_arena + s * c->arena_cap + p * pcap, used, hipMemcpyDeviceToHost)))
            return c->hipfail(e, "read name arena");
    }
    const std::vector<uint64_t> &roff = c->roff[s];
    // after a multi-GPU exchange (before pv_topn_x_view), this rank's regions only
    uint64_t i0 = 0, i1 = tcap;
    if (c->x_ranks > 1) {
        const uint32_t nreg = 1u << c->reg_log2, rsl = c->tcap_log2 - c->reg_log2;
        i0 = (uint64_t)(((uint64_t)c->x_rank * nreg + c->x_ranks - 1) / c->x_ranks) << rsl;
        i1 = (uint64_t)(((uint64_t)(c->x_rank + 1) * nreg + c->x_ranks - 1) / c->x_ranks) << rsl;
    }
    for (uint64_t i = i0; i < i1; i++) {
        if (!keys[i]) continue;
        // a purged region's survivors report count + the thetas its purges subtracted (the
        // frequent-items estimate, exact for a key no purge dropped)
        const uint64_t off = roff.empty() ? 0 : roff[(i >> (c->tcap_log2 - c->reg_log2))];
        TopRec r{keys[i], cnt[i] + off, std::string()};
        uint32_t m = PV_KEY_METRIC(keys[i]);
        if (m == TM_IPV4) {
            uint32_t ip = (uint32_t)keys[i];
            char b[20];
            snprintf(b, sizeof b, "%u.%u.%u.%u", ip & 0xff, (ip >> 8) & 0xff, (ip >> 16) & 0xff, ip >> 24);
            r.name = b;
        } else if (aux[i] && (aux[i] - 1) % pcap + 2 <= parts[(aux[i] - 1) / pcap].size()) {
            const std::vector<uint8_t> &arena = parts[(aux[i] - 1) / pcap];
            const uint64_t top = arena.size();
            uint64_t p = (aux[i] - 1) % pcap;
            uint32_t len = arena[p] | (arena[p + 1] << 8);
            if (p + 2 + len <= top) {
                if (m == TM_IPV6) {
                    char b[64];
                    inet_ntop(AF_INET6, &arena[p + 2], b, sizeof b);
                    r.name = b;
                } else if (m == TM_ECS && len == 17) {
                    // ECS client subnet text (inet_ntop, DnsAdditionalRecord.h:86,95)
                    char b[64];
                    inet_ntop(arena[p + 2] == 1 ? AF_INET : AF_INET6, &arena[p + 3], b, sizeof b);
                    r.name = b;
                } else {
                    r.name.assign((const char *)&arena[p + 2], len);
                }
            }
        }
        out.push_back(std::move(r));
    }
    auto it = c->remote_topn.find(s);
    if (it != c->remote_topn.end())
        for (auto &kv : it->second) out.push_back(TopRec{kv.first, kv.second.first, kv.second.second});
    return 0;
}

// Host-side metric of a top-N entry: its key's metric, or for Net v2 keys a metric per
// direction (TMH_V2_IP4 + dir, TMH_V2_IP6 + dir)
enum { TMH_V2_IP4 = 32, TMH_V2_IP6 = 36, TMH_V2_DNS = 64 }; // DNS v2: 64 + 4 * metric + dir
uint32_t host_metric(const pv_ctx *c, uint64_t key)
{
    if (PV_IS_V2_IP4(key)) return TMH_V2_IP4 + (uint32_t)((key >> 34) & 3);
    if (PV_IS_V2_IP6(key)) return TMH_V2_IP6 + (uint32_t)((key >> 53) & 3);
    // (v1 name keys carry a full 56-bit fingerprint: only a DNS v2 context holds v2 name keys)
    if (c->dns2_groups && PV_IS_V2_DKEY(key)) return TMH_V2_DNS + 4 * PV_KEY_METRIC(key) + (uint32_t)((key >> 53) & 3);
    return PV_KEY_METRIC(key);
}

// A finalised bucket (possibly the merge of several slots) on the host.
struct HostBucket {
    int64_t start_sec = 0;
    uint64_t period_length = 0;
    std::vector<uint64_t> sum;                           // PV_SUM_WORDS
    std::vector<int64_t> cpc;                            // PV_MIN_WORDS (min-merged)
    std::map<uint32_t, std::map<std::string, uint64_t>> tops; // metric -> name -> count
    std::vector<uint64_t> from_us, to_us;
    std::vector<double> ratio;
    std::vector<uint64_t> time2[3]; // DNS v2 per direction
    std::vector<double> ratio2[3];
    bool merged = false;
    // an exported bucket (pv_bucket) after an Aggregate::SUM merge: Quantile::_quantiles_sum
    // (src/Metrics.h:338-372), which the output prefers to the sketch's own quantiles, and the
    // Histogram values, which keep merging while the quantile sketches do not
    std::vector<uint64_t> qs_payload, qs_from, qs_to;
    std::vector<double> qs_ratio;
    bool hist_sep = false;
    std::vector<uint64_t> hfrom_us, hto_us;
    int64_t start_nsec = 0, end_sec = 0, end_nsec = 0;
    const std::vector<uint64_t> &hist_from() const { return hist_sep ? hfrom_us : from_us; }
    const std::vector<uint64_t> &hist_to() const { return hist_sep ? hto_us : to_us; }
    // the same for the v2 handlers, per direction: payload sizes (Net v2), transaction times and
    // size ratios (DNS v2) after a SUM merge, and the xact time histograms that keep merging
    std::vector<uint64_t> qs_payload2[3], qs_time2[3];
    std::vector<double> qs_ratio2[3];
    bool hist2_sep = false;
    std::vector<uint64_t> htime2[3];
    const std::vector<uint64_t> &hist_time2(uint32_t x) const { return hist2_sep ? htime2[x] : time2[x]; }
};

template <typename T>
std::vector<T> quantiles(std::vector<T> v)
{
    std::sort(v.begin(), v.end());
    std::vector<T> out;
    for (double r : {0.50, 0.90, 0.95, 0.99}) {
        uint64_t w = (uint64_t)std::ceil(r * (double)v.size());
        size_t idx = w == 0 ? 0 : (size_t)(w - 1);
        if (idx >= v.size()) idx = v.size() - 1;
        out.push_back(v[idx]);
    }
    return out;
}

// exact quantiles of the payload-size histogram with the KLL inclusive rank rule
std::vector<uint64_t> hist_quantiles(const uint64_t *h, size_t bins, uint64_t &n)
{
    n = 0;
    for (size_t i = 0; i < bins; i++) n += h[i];
    std::vector<uint64_t> out;
    if (!n) return out;
    for (double r : {0.50, 0.90, 0.95, 0.99}) {
        uint64_t w = (uint64_t)std::ceil(r * (double)n);
        if (w == 0) w = 1;
        uint64_t acc = 0;
        size_t i = 0;
        for (; i < bins; i++) { acc += h[i]; if (acc >= w) break; }
        out.push_back(std::min(i, bins - 1));
    }
    return out;
}

double cpc_estimate(const int64_t *t, bool merged)
{
    if (merged) {
        uint32_t c = 0;
        for (uint32_t i = 0; i < PV_CPC_COUPONS; i++) c += t[i] != PV_CPC_EMPTY;
        return icon11(c);
    }
    std::vector<std::pair<int64_t, uint32_t>> f;
    for (uint32_t i = 0; i < PV_CPC_COUPONS; i++)
        if (t[i] != PV_CPC_EMPTY) f.push_back({t[i], i});
    return cpc_hip(f);
}

// One handler's bucket over `slots` (merged: window_merged_json's fold, AbstractMetricsManager.h:601-647)
// The merged view's values of a set of DNS slots (pv_values_x_select; mask: bit per slot): per kind a stand-in list of the
// group's count whose histogram-point counts and maximum are the merged ones (each value at the
// point that bounds it, the largest replaced by the maximum), its quantiles set as overrides.
const std::vector<uint64_t> &hist_points();
void x_values_standin(pv_ctx *c, uint32_t mask, HostBucket &b)
{
    const std::vector<uint64_t> &pts = hist_points();
    for (auto &kv : c->xq) {
        if (kv.first.first != mask) continue;
        const uint32_t kind = kv.first.second;
        const XQuant &x = kv.second;
        std::vector<uint64_t> v;
        v.reserve(x.n);
        if (!x.cdf.empty()) {
            uint64_t prev = 0;
            for (size_t k = 0; k < pts.size(); k++) {
                for (uint64_t i = prev; i < x.cdf[k]; i++) v.push_back(pts[k]);
                prev = std::max(prev, x.cdf[k]);
            }
        }
        while (v.size() < x.n) v.push_back(x.max);
        if (!v.empty()) v.back() = x.max;
        auto dbl = [](const std::vector<uint64_t> &u) {
            std::vector<double> d(u.size());
            for (size_t i = 0; i < u.size(); i++) memcpy(&d[i], &u[i], 8);
            return d;
        };
        if (kind == XV_FROM_US) { b.from_us.insert(b.from_us.end(), v.begin(), v.end()); b.qs_from = x.q; }
        else if (kind == XV_TO_US) { b.to_us.insert(b.to_us.end(), v.begin(), v.end()); b.qs_to = x.q; }
        else if (kind == XV_RATIO) { auto d = dbl(v); b.ratio.insert(b.ratio.end(), d.begin(), d.end()); b.qs_ratio = dbl(x.q); }
        else if (kind >= XV2_TIME && kind < XV2_TIME + 3) { auto &t = b.time2[kind - XV2_TIME]; t.insert(t.end(), v.begin(), v.end()); b.qs_time2[kind - XV2_TIME] = x.q; }
        else if (kind >= XV2_RATIO && kind < XV2_RATIO + 3) {
            auto d = dbl(v);
            auto &t = b.ratio2[kind - XV2_RATIO];
            t.insert(t.end(), d.begin(), d.end());
            b.qs_ratio2[kind - XV2_RATIO] = dbl(x.q);
        }
    }
}

int load_bucket(pv_ctx *c, const std::vector<uint32_t> &slots, bool merged, int part, HostBucket &b)
{
    flush_fills(c);
    const Window &win = part == PART_NET ? c->net : c->dns;
    b.sum.assign(PV_SUM_WORDS, 0);
    b.cpc.assign(PV_MIN_WORDS, PV_CPC_EMPTY);
    b.merged = merged;
    // this handler's part of the slot's SUM and MIN words
    const size_t s0 = part == PART_NET ? 0 : PV_OFF_DNS, s1 = part == PART_NET ? PV_SUM_NET_WORDS : PV_SUM_WORDS;
    const size_t m0 = part == PART_NET ? 0 : PV_MIN_NET_WORDS, m1 = part == PART_NET ? PV_MIN_NET_WORDS : PV_MIN_WORDS;
    std::vector<uint64_t> sum(PV_SUM_WORDS);
    std::vector<int64_t> cpc(PV_MIN_WORDS);
    bool first = true;
    for (uint32_t s : slots) {
        hipError_t e;
        if (!hip_ok(e = hipMemcpyAsync(sum.data() + s0, c->d_sum + (uint64_t)s * PV_SUM_WORDS + s0, (s1 - s0) * 8,
                                       hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipMemcpyAsync(cpc.data() + m0, c->d_cpc + (uint64_t)s * PV_MIN_WORDS + m0, (m1 - m0) * 8,
                                       hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "read bucket");
        for (size_t i = s0; i < s1; i++) b.sum[i] += sum[i];
        // CPC union: a coupon is present if present in any bucket; for a single
        // bucket the first-occurrence order is kept for the HIP replay
        for (size_t i = m0; i < m1; i++) b.cpc[i] = std::min(b.cpc[i], cpc[i]);
        const SlotMeta &m = win.meta[s];
        b.period_length += m.read_only ? m.period_length : 0;
        if (first || m.start_sec < b.start_sec) { b.start_sec = m.start_sec; b.start_nsec = m.start_nsec; }
        if (m.end_sec > b.end_sec) { b.end_sec = m.end_sec; b.end_nsec = m.end_nsec; }
        first = false;
        if (!(c->x_ranks > 1 && c->x_view_on)) {
            std::vector<TopRec> recs;
            int rc = read_topn(c, s + (part == PART_DNS ? PV_SLOTS : 0), recs);
            if (rc) return rc;
            for (auto &r : recs) b.tops[host_metric(c, r.key)][r.name] += r.count;
        }
        if (part != PART_DNS) continue;
        const uint32_t sg = s | (c->gen[s] << 8);
        if (c->xq_on) continue; // (the merged view's values: after the loop, for the slot set)
        for (auto &v : c->xvals_host) {
            if (v.slot != sg) continue;
            if (v.kind == XV_FROM_US) b.from_us.push_back(v.bits);
            else if (v.kind == XV_TO_US) b.to_us.push_back(v.bits);
            else if (v.kind == XV_RATIO) { double d; memcpy(&d, &v.bits, 8); b.ratio.push_back(d); }
            else if (v.kind >= XV2_TIME && v.kind < XV2_TIME + 3) b.time2[v.kind - XV2_TIME].push_back(v.bits);
            else if (v.kind >= XV2_RATIO && v.kind < XV2_RATIO + 3) {
                double d;
                memcpy(&d, &v.bits, 8);
                b.ratio2[v.kind - XV2_RATIO].push_back(d);
            }
        }
    }
    uint32_t mask = 0;
    for (uint32_t sl : slots) mask |= 1u << sl;
    if (c->x_ranks > 1 && c->x_view_on) {
        // a multi-GPU merged view (pv_topn_x_view): every owner's leading entries of this slot set
        auto it = c->x_view.find(((uint32_t)part << 16) | mask);
        if (it != c->x_view.end())
            for (auto &kv : it->second) b.tops[host_metric(c, kv.first)][kv.second.second] += kv.second.first;
    }
    if (part == PART_DNS && c->xq_on) x_values_standin(c, mask, b);
    return 0;
}

// TopN::to_json (src/Metrics.h:577-590): the first topn_count items by estimate, cut at the
// first one below the topn_percentile_threshold quantile of those estimates (_get_threshold,
// :510-521, the KLL inclusive rank rule on them)
void top_json(Json &j, const char *key, const std::vector<std::pair<std::string, uint64_t>> &v0, size_t n, uint32_t pct)
{
    auto v = v0;
    std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
        if (a.second != b.second) return a.second > b.second;
        return a.first < b.first;
    });
    const size_t k = std::min(n, v.size());
    uint64_t thr = 0;
    if (k) {
        std::vector<uint64_t> est;
        for (size_t i = 0; i < k; i++) est.push_back(v[i].second);
        std::sort(est.begin(), est.end());
        const uint64_t w = (uint64_t)std::ceil((double)pct / 100.0 * (double)k);
        thr = est[w == 0 ? 0 : std::min<size_t>(w - 1, k - 1)];
    }
    j.key(key);
    j.arr();
    for (size_t i = 0; i < k && v[i].second >= thr; i++) {
        j.obj();
        j.key("name").str(v[i].first);
        j.key("estimate").u(v[i].second);
        j.end_obj();
    }
    j.end_arr();
}
std::vector<std::pair<std::string, uint64_t>> tops_of(const HostBucket &b, uint32_t metric)
{
    std::vector<std::pair<std::string, uint64_t>> v;
    auto it = b.tops.find(metric);
    if (it != b.tops.end())
        for (auto &kv : it->second) v.push_back(kv);
    return v;
}
std::vector<std::pair<std::string, uint64_t>> dense_tops(const uint64_t *t, size_t bins, int kind)
{
    std::vector<std::pair<std::string, uint64_t>> v;
    for (size_t i = 0; i < bins; i++) {
        if (!t[i]) continue;
        std::string name;
        if (kind == 0) name = std::to_string(i);
        else {
            auto &m = kind == 1 ? qtype_names() : rcode_names();
            auto it = m.find((uint16_t)i);
            name = it != m.end() ? it->second : std::to_string(i);
        }
        v.push_back({name, t[i]});
    }
    return v;
}

// Histogram::to_json (src/Metrics.h:193-262) over exact values: split points are the distinct
// uint64 values of 10^(b/18) * 10^e, e in [-9, 18), b in [0, 18); a point is listed when the
// inclusive PMF interval that ends at it holds a value, with the inclusive CDF times n (a
// double, as KLL's normalized rank times get_n()); "+Inf" closes with n
const std::vector<uint64_t> &hist_points()
{
    static const std::vector<uint64_t> pts = [] {
        std::vector<uint64_t> p;
        for (int e = -9; e < 18; e++)
            for (int k = 0; k < 18; k++) {
                const uint64_t x = static_cast<uint64_t>(std::pow(10.0, static_cast<float>(k) / 18) * std::pow(10.0, e));
                if (p.empty() || p.back() != x) p.push_back(x);
            }
        return p;
    }();
    return pts;
}
void hist_json(Json &j, const char *key, std::vector<uint64_t> v)
{
    if (v.empty()) return;
    const std::vector<uint64_t> &pts = hist_points();
    std::sort(v.begin(), v.end());
    const double n = (double)v.size();
    j.key(key).obj();
    j.key("buckets").obj();
    uint64_t prev = 0;
    for (uint64_t x : pts) {
        const uint64_t c = (uint64_t)(std::upper_bound(v.begin(), v.end(), x) - v.begin());
        if (c != prev) j.key(std::to_string(x)).d(((double)c / n) * n);
        prev = c;
    }
    j.key("+Inf").d(1.0 * n);
    j.end_obj();
    j.end_obj();
}

template <typename T>
void quant_json(Json &j, const char *key, const std::vector<T> &v, const std::vector<T> *qsum = nullptr)
{
    if (v.empty()) return;
    auto q = qsum && !qsum->empty() ? *qsum : quantiles(v);
    const char *names[4] = {"p50", "p90", "p95", "p99"};
    j.key(key);
    j.obj();
    for (int i = 0; i < 4; i++) {
        j.key(names[i]);
        if constexpr (std::is_floating_point<T>::value) j.d(q[i]);
        else j.u((uint64_t)q[i]);
    }
    j.end_obj();
}

void net_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET];
    size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("events").u(n[NC_EVENTS]);
    j.key("deep_samples").u(n[NC_SAMPLES]);
    if (c->net_groups & PV_NET_COUNTERS) {
        j.key("udp").u(n[NC_UDP]);
        j.key("tcp").u(n[NC_TCP]);
        j.key("protocol").obj(); j.key("tcp").obj(); j.key("syn").u(n[NC_SYN]); j.end_obj(); j.end_obj();
        j.key("other_l4").u(n[NC_OTHER]);
        j.key("ipv4").u(n[NC_V4]);
        j.key("ipv6").u(n[NC_V6]);
        j.key("in").u(n[NC_IN]);
        j.key("out").u(n[NC_OUT]);
        j.key("unknown_dir").u(n[NC_UNK]);
        j.key("total").u(n[NC_TOTAL]);
        j.key("filtered").u(n[NC_FILTERED]);
    }
    if (c->net_groups & PV_NET_CARDINALITY) {
        j.key("cardinality").obj();
        j.key("src_ips_in").i(lround(cpc_estimate(&b.cpc[CPC_SRC * PV_CPC_COUPONS], b.merged)));
        j.key("dst_ips_out").i(lround(cpc_estimate(&b.cpc[CPC_DST * PV_CPC_COUPONS], b.merged)));
        j.end_obj();
    }
    if (c->net_groups & PV_NET_TOP_IPS) {
        top_json(j, "top_ipv4", tops_of(b, TM_IPV4), topn, pct);
        top_json(j, "top_ipv6", tops_of(b, TM_IPV6), topn, pct);
    }
    if (c->net_groups & PV_NET_TOP_GEO) {
        j.key("top_geoLoc").arr(); j.end_arr();
        j.key("top_ASN").arr(); j.end_arr();
    }
    uint64_t cnt;
    auto q = hist_quantiles(&b.sum[PV_OFF_PAYLOAD], PV_PAYLOAD_BINS, cnt);
    if (!b.qs_payload.empty()) q = b.qs_payload;
    if (cnt) {
        j.key("payload_size").obj();
        j.key("p50").u(q[0]); j.key("p90").u(q[1]); j.key("p95").u(q[2]); j.key("p99").u(q[3]);
        j.end_obj();
    }
}

// NetworkMetricsBucket::to_json, Net v2 (src/handlers/net/v2/NetStreamHandler.cpp:436-484):
// base event counts, `filtered_packets`, then one object per direction the bucket has seen
// (the reference creates a direction's entry on its first packet)
void net2_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET2];
    const uint32_t g = c->net2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("observed_packets").u(n[N2_EVENTS]);
    j.key("deep_sampled_packets").u(n[N2_SAMPLES]);
    if (g & PV_N2G_COUNTERS) j.key("filtered_packets").u(n[N2_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    for (uint32_t d = 0; d < 3; d++) {
        const uint64_t *dc = n + N2_DIR + 8 * d;
        if (!dc[N2_TOTAL]) continue;
        j.key(dirs[d]).obj();
        if (g & PV_N2G_COUNTERS) {
            j.key("udp_packets").u(dc[N2_UDP]);
            j.key("tcp_packets").u(dc[N2_TCP]);
            j.key("other_l4_packets").u(dc[N2_OTHER]);
            j.key("ipv4_packets").u(dc[N2_V4]);
            j.key("ipv6_packets").u(dc[N2_V6]);
            j.key("tcp").obj(); j.key("syn_packets").u(dc[N2_SYN]); j.end_obj();
            j.key("total_packets").u(dc[N2_TOTAL]);
        }
        if (g & PV_N2G_CARDINALITY) {
            j.key("cardinality").obj();
            j.key("ips").i(lround(cpc_estimate(&b.cpc[(CPC_V2 + d) * PV_CPC_COUPONS], b.merged)));
            j.end_obj();
        }
        if (g & PV_N2G_TOP_IPS) {
            top_json(j, "top_ipv4_packets", tops_of(b, TMH_V2_IP4 + d), topn, pct);
            top_json(j, "top_ipv6_packets", tops_of(b, TMH_V2_IP6 + d), topn, pct);
        }
        if (g & PV_N2G_TOP_GEO) {
            j.key("top_geo_loc_packets").arr(); j.end_arr();
            j.key("top_asn_packets").arr(); j.end_arr();
        }
        if (g & PV_N2G_QUANTILES) {
            uint64_t cnt;
            auto q = hist_quantiles(&b.sum[PV_OFF_PAYLOAD2 + d * PV_PAYLOAD_BINS], PV_PAYLOAD_BINS, cnt);
            if (cnt && !b.qs_payload2[d].empty()) q = b.qs_payload2[d];
            if (cnt) {
                j.key("payload_size_bytes").obj();
                j.key("p50").u(q[0]); j.key("p90").u(q[1]); j.key("p95").u(q[2]); j.key("p99").u(q[3]);
                j.end_obj();
            }
        }
        j.end_obj();
    }
}

// DnsMetricsBucket::to_json, DNS v2 (src/handlers/dns/v2/DnsStreamHandler.cpp:678-757): base
// event counts (the DNS pass's event counters), `filtered_packets`, then per transaction
// direction the bucket has set up: counters, qname cardinality and the top / quantile groups
void dns2_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    const uint32_t g = c->dns2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("observed_packets").u(d[DC_EVENTS]);
    j.key("deep_sampled_packets").u(d[DC_SAMPLES]);
    if (g & PV_DNS2_COUNTERS) j.key("filtered_packets").u(d[DC_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    for (uint32_t x = 0; x < 3; x++) {
        const uint64_t *c2 = &b.sum[PV_OFF_DNS2 + x * PV_DNS2_CTRS];
        if (!c2[D2_SEEN]) continue;
        auto tops = [&](uint32_t metric) { return tops_of(b, TMH_V2_DNS + 4 * metric + x); };
        j.key(dirs[x]).obj();
        if (g & PV_DNS2_COUNTERS) {
            const std::pair<const char *, uint64_t> ctr[] = {
                {"xacts", c2[D2_XACTS]}, {"udp_xacts", c2[D2_UDP]}, {"tcp_xacts", c2[D2_TCP]}, {"dot_xacts", c2[D2_DOT]},
                {"doh_xacts", c2[D2_DOH]}, {"dnscrypt_udp_xacts", c2[D2_CRYPT_UDP]}, {"dnscrypt_tcp_xacts", c2[D2_CRYPT_TCP]},
                {"doq_xacts", c2[D2_DOQ]},
                {"ipv4_xacts", c2[D2_V4]}, {"ipv6_xacts", c2[D2_V6]}, {"nxdomain_xacts", c2[D2_NX]}, {"ecs_xacts", c2[D2_ECS]},
                {"refused_xacts", c2[D2_REFUSED]}, {"srvfail_xacts", c2[D2_SRVFAIL]}, {"noerror_xacts", c2[D2_NOERROR]},
                {"nodata_xacts", c2[D2_NODATA]}, {"authenticated_data_xacts", c2[D2_AD]},
                {"authoritative_answer_xacts", c2[D2_AA]}, {"checking_disabled_xacts", c2[D2_CD]},
                {"timeout_queries", c2[D2_TIMEOUT]}, {"orphan_responses", c2[D2_ORPHAN]}};
            for (auto &kv : ctr) j.key(kv.first).u(kv.second);
        }
        if (g & PV_DNS2_CARDINALITY) {
            j.key("cardinality").obj();
            j.key("qname").i(lround(cpc_estimate(&b.cpc[(CPC_QNAME2 + x) * PV_CPC_COUPONS], b.merged)));
            j.end_obj();
        }
        if (g & PV_DNS2_TOP_PORTS)
            top_json(j, "top_udp_ports_xacts", dense_tops(&b.sum[PV_OFF_PORT2 + x * PV_PORT_BINS], PV_PORT_BINS, 0), topn, pct);
        if (g & PV_DNS2_TOP_ECS) {
            // geo / ASN of the subnet need a MaxMind database; none is enabled (HandlerModulePlugin::city/asn)
            j.key("top_geo_loc_ecs_xacts").arr(); j.end_arr();
            j.key("top_asn_ecs_xacts").arr(); j.end_arr();
            top_json(j, "top_ecs_xacts", tops(TM_ECS), topn, pct);
        }
        if (g & PV_DNS2_TOP_RCODES) {
            top_json(j, "top_nxdomain_xacts", tops(TM_NX), topn, pct);
            top_json(j, "top_refused_xacts", tops(TM_REFUSED), topn, pct);
            top_json(j, "top_srvfail_xacts", tops(TM_SRVFAIL), topn, pct);
            top_json(j, "top_nodata_xacts", tops(TM_NODATA), topn, pct);
            top_json(j, "top_noerror_xacts", tops(TM_NOERROR), topn, pct);
            top_json(j, "top_rcode_xacts", dense_tops(&b.sum[PV_OFF_RCODE2 + x * PV_RCODE_BINS], PV_RCODE_BINS, 2), topn, pct);
        }
        if (g & PV_DNS2_TOP_QNAMES) {
            top_json(j, "top_qname2_xacts", tops(TM_QNAME2), topn, pct);
            top_json(j, "top_qname3_xacts", tops(TM_QNAME3), topn, pct);
        }
        if (g & PV_DNS2_TOP_SIZE) {
            top_json(j, "top_response_bytes", tops(TM_SIZED), topn, pct);
            quant_json(j, "response_query_size_ratio", b.ratio2[x], &b.qs_ratio2[x]);
        }
        if (g & PV_DNS2_TOP_QTYPES)
            top_json(j, "top_qtype_xacts", dense_tops(&b.sum[PV_OFF_QTYPE2 + x * PV_QTYPE_BINS], PV_QTYPE_BINS, 1), topn, pct);
        if (g & PV_DNS2_XACT_TIMES) {
            quant_json(j, "xact_time_us", b.time2[x], &b.qs_time2[x]);
            hist_json(j, "xact_histogram_us", b.hist_time2(x));
            top_json(j, "top_slow_xacts", tops(TM_SLOW_OUT), topn, pct);
        }
        j.end_obj();
    }
}

void dns_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    uint32_t g = c->dns_groups;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("wire_packets").obj();
    j.key("events").u(d[DC_EVENTS]);
    j.key("deep_samples").u(d[DC_SAMPLES]);
    if (g & PV_DNS_COUNTERS) {
        j.key("queries").u(d[DC_QUERIES]);
        j.key("replies").u(d[DC_REPLIES]);
        j.key("tcp").u(d[DC_TCP]);
        j.key("udp").u(d[DC_UDP]);
        j.key("ipv4").u(d[DC_V4]);
        j.key("ipv6").u(d[DC_V6]);
        j.key("nxdomain").u(d[DC_NX]);
        j.key("refused").u(d[DC_REFUSED]);
        j.key("srvfail").u(d[DC_SRVFAIL]);
        j.key("noerror").u(d[DC_NOERROR]);
        j.key("nodata").u(d[DC_NODATA]);
        j.key("total").u(d[DC_TOTAL]);
        j.key("filtered").u(d[DC_FILTERED]);
        if (g & PV_DNS_TOP_ECS) j.key("query_ecs").u(d[DC_QECS]);
    }
    j.end_obj();
    if (g & PV_DNS_CARDINALITY) {
        j.key("cardinality").obj();
        j.key("qname").i(lround(cpc_estimate(&b.cpc[CPC_QNAME * PV_CPC_COUPONS], b.merged)));
        j.end_obj();
    }
    if (g & PV_DNS_TRANSACTIONS) {
        j.key("xact").obj();
        j.key("counts").obj(); j.key("total").u(d[DC_XTOTAL]); j.key("timed_out").u(d[DC_XTIMEOUT]); j.end_obj();
        j.key("in").obj();
        j.key("total").u(d[DC_XIN]);
        top_json(j, "top_slow", tops_of(b, TM_SLOW_IN), topn, pct);
        if (g & PV_DNS_QUANTILES) quant_json(j, "quantiles_us", b.to_us, &b.qs_to);
        if (g & PV_DNS_HISTOGRAMS) hist_json(j, "histogram_us", b.hist_to());
        j.end_obj();
        j.key("out").obj();
        j.key("total").u(d[DC_XOUT]);
        top_json(j, "top_slow", tops_of(b, TM_SLOW_OUT), topn, pct);
        if (g & PV_DNS_QUANTILES) quant_json(j, "quantiles_us", b.from_us, &b.qs_from);
        if (g & PV_DNS_HISTOGRAMS) hist_json(j, "histogram_us", b.hist_from());
        j.end_obj();
        if ((g & PV_DNS_QUANTILES) && !b.ratio.empty()) { j.key("ratio").obj(); quant_json(j, "quantiles", b.ratio, &b.qs_ratio); j.end_obj(); }
        j.end_obj();
    }
    if (g & PV_DNS_TOP_PORTS) top_json(j, "top_udp_ports", dense_tops(&b.sum[PV_OFF_PORT], PV_PORT_BINS, 0), topn, pct);
    if (g & PV_DNS_TOP_ECS) {
        // geo / ASN of the subnet need a MaxMind database; none is enabled (HandlerModulePlugin::city/asn)
        j.key("top_geoLoc_ecs").arr(); j.end_arr();
        j.key("top_asn_ecs").arr(); j.end_arr();
        top_json(j, "top_query_ecs", tops_of(b, TM_ECS), topn, pct);
    }
    if (g & PV_DNS_TOP_QNAMES) {
        top_json(j, "top_qname2", tops_of(b, TM_QNAME2), topn, pct);
        top_json(j, "top_qname3", tops_of(b, TM_QNAME3), topn, pct);
        top_json(j, "top_nxdomain", tops_of(b, TM_NX), topn, pct);
        top_json(j, "top_refused", tops_of(b, TM_REFUSED), topn, pct);
        top_json(j, "top_srvfail", tops_of(b, TM_SRVFAIL), topn, pct);
        top_json(j, "top_nodata", tops_of(b, TM_NODATA), topn, pct);
        if (g & PV_DNS_TOP_QNAMES_DETAILS) {
            top_json(j, "top_qname_by_resp_bytes", tops_of(b, TM_SIZED), topn, pct);
            top_json(j, "top_noerror", tops_of(b, TM_NOERROR), topn, pct);
        }
    }
    top_json(j, "top_rcode", dense_tops(&b.sum[PV_OFF_RCODE], PV_RCODE_BINS, 2), topn, pct);
    top_json(j, "top_qtype", dense_tops(&b.sum[PV_OFF_QTYPE], PV_QTYPE_BINS, 1), topn, pct);
}

// ---- Prometheus exposition (window_single_prometheus, src/AbstractMetricsManager.h:506-531)
// Metric text as the reference's primitives write it (src/Metrics.cpp:15-20,75-80,120-155;
// src/Metrics.h:264-289,416-448,614-691): "# HELP <schema>_<names> <desc>", "# TYPE ...", then
// samples named <schema>_<names>[_suffix]{static labels, then the added labels, each set in key
// order}. Numbers go through an ostream, as the reference's do (doubles with precision 6).
// Rates are timer-driven and not kept by this handler: an empty Rate writes nothing.
using PromLabels = std::map<std::string, std::string>;
std::mutex g_static_mu;
PromLabels g_static_labels; // Metric::_static_labels (Metric::add_static_label)

struct Prom {
    std::ostringstream o;
    PromLabels add;
    std::string lbl(const PromLabels &a) const
    {
        std::string t = "{";
        {
            std::lock_guard<std::mutex> g(g_static_mu);
            for (auto &kv : g_static_labels) t += kv.first + "=\"" + kv.second + "\",";
        }
        for (auto &kv : a) t += kv.first + "=\"" + kv.second + "\",";
        if (t.back() == ',') t.pop_back();
        return t + "}";
    }
    void head(const std::string &name, const char *desc, const char *type)
    {
        o << "# HELP " << name << ' ' << desc << '\n' << "# TYPE " << name << ' ' << type << '\n';
    }
    template <typename V>
    void gauge(const std::string &name, const char *desc, V v)
    {
        head(name, desc, "gauge");
        o << name << lbl(add) << ' ' << v << '\n';
    }
    // Quantile::to_prometheus: p50..p99, _sum = the sketch's max item, _count = n
    template <typename T>
    void summary(const std::string &name, const char *desc, const std::vector<T> &q, T max_item, uint64_t n)
    {
        if (q.empty()) return;
        head(name, desc, "summary");
        static const char *qs[4] = {"0.5", "0.9", "0.95", "0.99"};
        for (int i = 0; i < 4; i++) {
            PromLabels l(add);
            l["quantile"] = qs[i];
            o << name << lbl(l) << ' ' << q[i] << '\n';
        }
        o << name << "_sum" << lbl(add) << ' ' << max_item << '\n';
        o << name << "_count" << lbl(add) << ' ' << n << '\n';
    }
    // TopN::to_prometheus: the to_json selection, one sample per item labelled item_key=name
    void topn(const std::string &name, const char *item_key, const char *desc,
              const std::vector<std::pair<std::string, uint64_t>> &v0, size_t n, uint32_t pct)
    {
        auto v = v0;
        std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
            if (a.second != b.second) return a.second > b.second;
            return a.first < b.first;
        });
        const size_t k = std::min(n, v.size());
        if (!k) return;
        std::vector<uint64_t> est;
        for (size_t i = 0; i < k; i++) est.push_back(v[i].second);
        std::sort(est.begin(), est.end());
        const uint64_t w = (uint64_t)std::ceil((double)pct / 100.0 * (double)k);
        const uint64_t thr = est[w == 0 ? 0 : std::min<size_t>(w - 1, k - 1)];
        head(name, desc, "gauge");
        PromLabels l(add);
        for (size_t i = 0; i < k && v[i].second >= thr; i++) {
            l[item_key] = v[i].first;
            o << name << lbl(l) << ' ' << v[i].second << '\n';
        }
    }
    // Histogram::to_prometheus over exact values (the split points of hist_json)
    void histogram(const std::string &name, const char *desc, std::vector<uint64_t> v)
    {
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        head(name, desc, "histogram");
        const double n = (double)v.size();
        uint64_t prev = 0;
        for (uint64_t x : hist_points()) {
            const uint64_t c = (uint64_t)(std::upper_bound(v.begin(), v.end(), x) - v.begin());
            if (c != prev) {
                PromLabels l(add);
                l["le"] = std::to_string(x);
                o << name << "_bucket" << lbl(l) << ' ' << ((double)c / n) * n << '\n';
            }
            prev = c;
        }
        PromLabels l(add);
        l["le"] = "+Inf";
        o << name << "_bucket" << lbl(l) << ' ' << 1.0 * n << '\n';
        o << name << "_count" << lbl(add) << ' ' << v.size() << '\n';
    }
};

// ---- OpenTelemetry (window_single_opentelemetry, src/AbstractMetricsManager.h:533-575): the
// metrics the reference's primitives add to a ScopeMetrics (src/Metrics.cpp:22-36,82-96;
// src/Metrics.h:289-327,450-481,523-533,693-769), as protobuf wire bytes of the ScopeMetrics
// fields they fill (repeated `metrics`, field 2), serialized as protobuf does: fields in
// number order, proto3 defaults omitted, oneof members always written, packed repeated
// scalars. Messages of opentelemetry-proto metrics/v1 (the reference links
// opentelemetry-cpp 1.17.0's opentelemetry_proto; not vendored, field numbers restated):
// Metric{name 1, description 2, gauge 5, histogram 9, summary 11}; Gauge/Summary/Histogram
// {data_points 1; Histogram.aggregation_temporality 2}; NumberDataPoint{start 2, time 3,
// as_int 6, attributes 7}; SummaryDataPoint{start 2, time 3, quantile_values 6, attributes 7};
// ValueAtQuantile{quantile 1, value 2}; HistogramDataPoint{start 2, time 3, count 4,
// bucket_counts 6, explicit_bounds 7, attributes 9}; KeyValue{key 1, value 2};
// AnyValue{string_value 1}. Attributes are the added labels only (no static labels).
struct Pb {
    std::string s;
    void varint(uint64_t v)
    {
        while (v >= 0x80) { s.push_back((char)(uint8_t)(v | 0x80)); v >>= 7; }
        s.push_back((char)(uint8_t)v);
    }
    void tag(uint32_t f, uint32_t wt) { varint((uint64_t)f << 3 | wt); }
    void bytes(uint32_t f, const std::string &v) { tag(f, 2); varint(v.size()); s += v; }
    void str(uint32_t f, const std::string &v) { if (!v.empty()) bytes(f, v); }
    void fx64(uint32_t f, uint64_t v, bool always = false)
    {
        if (!v && !always) return;
        tag(f, 1);
        s.append(reinterpret_cast<const char *>(&v), 8);
    }
    void dbl(uint32_t f, double v)
    {
        uint64_t u;
        memcpy(&u, &v, 8);
        fx64(f, u);
    }
    void enm(uint32_t f, uint32_t v) { if (v) { tag(f, 0); varint(v); } }
};
struct Otlp {
    Pb out; // ScopeMetrics fields
    PromLabels add;
    uint64_t t0 = 0, t1 = 0;
    std::string attrs(uint32_t f, const PromLabels &l) const
    {
        Pb p;
        for (auto &kv : l) {
            Pb any, kvm;
            any.bytes(1, kv.second); // oneof string_value: written even when empty
            kvm.str(1, kv.first);
            kvm.bytes(2, any.s);
            p.bytes(f, kvm.s);
        }
        return p.s;
    }
    std::string number_point(const PromLabels &l, int64_t v) const
    {
        Pb d;
        d.fx64(2, t0);
        d.fx64(3, t1);
        d.fx64(6, (uint64_t)v, true); // oneof as_int
        d.s += attrs(7, l);
        return d.s;
    }
    void metric(const std::string &name, const char *desc, uint32_t field, const std::string &data, bool has_data = true)
    {
        Pb m;
        m.str(1, name);
        m.str(2, desc);
        if (has_data) m.bytes(field, data);
        out.bytes(2, m.s);
    }
    // Counter / Cardinality: a gauge of one int point
    template <typename V>
    void gauge(const std::string &name, const char *desc, V v)
    {
        Pb g;
        g.bytes(1, number_point(add, (int64_t)v));
        metric(name, desc, 5, g.s);
    }
    // Quantile: a summary point with the four quantiles (no count / sum, as the reference)
    template <typename T>
    void summary(const std::string &name, const char *desc, const std::vector<T> &q, T, uint64_t)
    {
        if (q.empty()) return;
        static const double fr[4] = {0.50, 0.90, 0.95, 0.99};
        Pb d;
        d.fx64(2, t0);
        d.fx64(3, t1);
        for (int i = 0; i < 4; i++) {
            Pb qv;
            qv.dbl(1, fr[i]);
            qv.dbl(2, (double)q[i]);
            d.bytes(6, qv.s);
        }
        d.s += attrs(7, add);
        Pb sm;
        sm.bytes(1, d.s);
        metric(name, desc, 11, sm.s);
    }
    // TopN: one gauge point per reported item (items with an empty name are skipped)
    void topn(const std::string &name, const char *item_key, const char *desc,
              const std::vector<std::pair<std::string, uint64_t>> &v0, size_t n, uint32_t pct)
    {
        auto v = v0;
        std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
            if (a.second != b.second) return a.second > b.second;
            return a.first < b.first;
        });
        const size_t k = std::min(n, v.size());
        if (!k) return;
        std::vector<uint64_t> est;
        for (size_t i = 0; i < k; i++) est.push_back(v[i].second);
        std::sort(est.begin(), est.end());
        const uint64_t w = (uint64_t)std::ceil((double)pct / 100.0 * (double)k);
        const uint64_t thr = est[w == 0 ? 0 : std::min<size_t>(w - 1, k - 1)];
        PromLabels l(add);
        Pb g;
        bool any = false;
        for (size_t i = 0; i < k && v[i].second >= thr; i++) {
            if (v[i].first.empty()) continue;
            l[item_key] = v[i].first;
            g.bytes(1, number_point(l, (int64_t)v[i].second));
            any = true;
        }
        metric(name, desc, 5, g.s, any);
    }
    // Histogram: bounds at the listed split points, bucket_counts as the reference computes
    // them (static_cast<uint64_t>(cdf) * n: n where the CDF reached 1, else 0)
    void histogram(const std::string &name, const char *desc, std::vector<uint64_t> v)
    {
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        const uint64_t n = v.size();
        std::vector<uint64_t> cnt;
        std::vector<double> bnd;
        uint64_t prev = 0;
        for (uint64_t x : hist_points()) {
            const uint64_t c = (uint64_t)(std::upper_bound(v.begin(), v.end(), x) - v.begin());
            if (c != prev) {
                bnd.push_back((double)x);
                cnt.push_back(static_cast<uint64_t>((double)c / (double)n) * n);
            }
            prev = c;
        }
        Pb d;
        d.fx64(2, t0);
        d.fx64(3, t1);
        d.fx64(4, n);
        d.tag(6, 2);
        d.varint(cnt.size() * 8);
        d.s.append(reinterpret_cast<const char *>(cnt.data()), cnt.size() * 8);
        d.tag(7, 2);
        d.varint(bnd.size() * 8);
        d.s.append(reinterpret_cast<const char *>(bnd.data()), bnd.size() * 8);
        d.s += attrs(9, add);
        Pb h;
        h.bytes(1, d.s);
        h.enm(2, 2); // AGGREGATION_TEMPORALITY_CUMULATIVE
        metric(name, desc, 9, h.s);
    }
};

// NetworkMetricsBucket::to_prometheus (src/handlers/net/v1/NetStreamHandler.cpp:332-388);
// names and descriptions from NetStreamHandler.h:81-127
template <class Sink>
void net_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET];
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    p.gauge("packets_events", "Total packets events generated", n[NC_EVENTS]);
    p.gauge("packets_deep_samples", "Total packets that were sampled for deep inspection", n[NC_SAMPLES]);
    if (c->net_groups & PV_NET_COUNTERS) {
        p.gauge("packets_udp", "Count of UDP packets", n[NC_UDP]);
        p.gauge("packets_tcp", "Count of TCP packets", n[NC_TCP]);
        p.gauge("packets_protocol_tcp_syn", "Count of TCP SYN packets", n[NC_SYN]);
        p.gauge("packets_other_l4", "Count of packets which are not UDP or TCP", n[NC_OTHER]);
        p.gauge("packets_ipv4", "Count of IPv4 packets", n[NC_V4]);
        p.gauge("packets_ipv6", "Count of IPv6 packets", n[NC_V6]);
        p.gauge("packets_in", "Count of total ingress packets", n[NC_IN]);
        p.gauge("packets_out", "Count of total egress packets", n[NC_OUT]);
        p.gauge("packets_unknown_dir", "Count of total unknown direction packets", n[NC_UNK]);
        p.gauge("packets_total", "Count of total packets matching the configured filter(s)", n[NC_TOTAL]);
        p.gauge("packets_filtered", "Count of total packets that did not match the configured filter(s) (if any)", n[NC_FILTERED]);
    }
    if (c->net_groups & PV_NET_CARDINALITY) {
        p.gauge("packets_cardinality_src_ips_in", "Source IP cardinality", lround(cpc_estimate(&b.cpc[CPC_SRC * PV_CPC_COUPONS], b.merged)));
        p.gauge("packets_cardinality_dst_ips_out", "Destination IP cardinality", lround(cpc_estimate(&b.cpc[CPC_DST * PV_CPC_COUPONS], b.merged)));
    }
    if (c->net_groups & PV_NET_TOP_IPS) {
        p.topn("packets_top_ipv4", "ipv4", "Top IPv4 IP addresses", tops_of(b, TM_IPV4), topn, pct);
        p.topn("packets_top_ipv6", "ipv6", "Top IPv6 IP addresses", tops_of(b, TM_IPV6), topn, pct);
    }
    // top_geo: no MaxMind database, the TopNs stay empty and write nothing
    uint64_t cnt;
    const uint64_t *h = &b.sum[PV_OFF_PAYLOAD];
    auto q = hist_quantiles(h, PV_PAYLOAD_BINS, cnt);
    if (!b.qs_payload.empty() && cnt) q = b.qs_payload;
    uint64_t mx = 0;
    for (size_t i = 0; i < PV_PAYLOAD_BINS; i++)
        if (h[i]) mx = i;
    p.template summary<uint64_t>("packets_payload_size", "Quantiles of payload sizes, in bytes", q, mx, cnt);
}

// DnsMetricsBucket::to_prometheus (src/handlers/dns/v1/DnsStreamHandler.cpp:1139-1238);
// names and descriptions from DnsStreamHandler.h:116-171
template <class Sink>
void dns_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    const uint32_t g = c->dns_groups;
    p.gauge("dns_wire_packets_events", "Total DNS wire packets events", d[DC_EVENTS]);
    p.gauge("dns_wire_packets_deep_samples", "Total DNS wire packets that were sampled for deep inspection", d[DC_SAMPLES]);
    if (g & PV_DNS_COUNTERS) {
        p.gauge("dns_wire_packets_queries", "Total DNS wire packets flagged as query (ingress and egress)", d[DC_QUERIES]);
        p.gauge("dns_wire_packets_replies", "Total DNS wire packets flagged as reply (ingress and egress)", d[DC_REPLIES]);
        p.gauge("dns_wire_packets_tcp", "Total DNS wire packets received over TCP (ingress and egress)", d[DC_TCP]);
        p.gauge("dns_wire_packets_udp", "Total DNS wire packets received over UDP (ingress and egress)", d[DC_UDP]);
        p.gauge("dns_wire_packets_ipv4", "Total DNS wire packets received over IPv4 (ingress and egress)", d[DC_V4]);
        p.gauge("dns_wire_packets_ipv6", "Total DNS wire packets received over IPv6 (ingress and egress)", d[DC_V6]);
        p.gauge("dns_wire_packets_nxdomain", "Total DNS wire packets flagged as reply with response code NXDOMAIN (ingress and egress)", d[DC_NX]);
        p.gauge("dns_wire_packets_refused", "Total DNS wire packets flagged as reply with response code REFUSED (ingress and egress)", d[DC_REFUSED]);
        p.gauge("dns_wire_packets_srvfail", "Total DNS wire packets flagged as reply with response code SRVFAIL (ingress and egress)", d[DC_SRVFAIL]);
        p.gauge("dns_wire_packets_noerror", "Total DNS wire packets flagged as reply with response code NOERROR (ingress and egress)", d[DC_NOERROR]);
        p.gauge("dns_wire_packets_nodata", "Total DNS wire packets flagged as reply with response code NOERROR and no answer section data (ingress and egress)", d[DC_NODATA]);
        p.gauge("dns_wire_packets_total", "Total DNS wire packets matching the configured filter(s)", d[DC_TOTAL]);
        p.gauge("dns_wire_packets_filtered", "Total DNS wire packets seen that did not match the configured filter(s) (if any)", d[DC_FILTERED]);
    }
    if (g & PV_DNS_CARDINALITY)
        p.gauge("dns_cardinality_qname", "Cardinality of unique QNAMES, both ingress and egress", lround(cpc_estimate(&b.cpc[CPC_QNAME * PV_CPC_COUPONS], b.merged)));
    auto vmax = [](const auto &v) { return v.empty() ? 0 : *std::max_element(v.begin(), v.end()); };
    if (g & PV_DNS_TRANSACTIONS) {
        p.gauge("dns_xact_counts_total", "Total DNS transactions (query/reply pairs)", d[DC_XTOTAL]);
        p.gauge("dns_xact_counts_timed_out", "Total number of DNS transactions that timed out", d[DC_XTIMEOUT]);
        p.gauge("dns_xact_in_total", "Total ingress DNS transactions (host is server)", d[DC_XIN]);
        p.topn("dns_xact_in_top_slow", "qname", "Top QNAMES in transactions where host is the server and transaction speed is slower than p90",
               tops_of(b, TM_SLOW_IN), topn, pct);
        if (g & PV_DNS_QUANTILES) {
            if (!b.from_us.empty())
                p.template summary<uint64_t>("dns_xact_out_quantiles_us", "Quantiles of transaction timing (query/reply pairs) when host is client, in microseconds",
                                    b.qs_from.empty() ? quantiles(b.from_us) : b.qs_from, vmax(b.from_us), b.from_us.size());
            if (!b.to_us.empty())
                p.template summary<uint64_t>("dns_xact_in_quantiles_us", "Quantiles of transaction timing (query/reply pairs) when host is server, in microseconds",
                                    b.qs_to.empty() ? quantiles(b.to_us) : b.qs_to, vmax(b.to_us), b.to_us.size());
            if (!b.ratio.empty())
                p.template summary<double>("dns_xact_ratio_quantiles", "Quantiles of ratio of packet sizes in a DNS transaction (reply/query)",
                                  b.qs_ratio.empty() ? quantiles(b.ratio) : b.qs_ratio, vmax(b.ratio), b.ratio.size());
        }
        if (g & PV_DNS_HISTOGRAMS) {
            p.histogram("dns_xact_out_histogram_us", "Histogram of transaction timing (query/reply pairs) when host is client, in microseconds", b.hist_from());
            p.histogram("dns_xact_in_histogram_us", "Histogram of transaction timing (query/reply pairs) when host is server, in microseconds", b.hist_to());
        }
        p.gauge("dns_xact_out_total", "Total egress DNS transactions (host is client)", d[DC_XOUT]);
        p.topn("dns_xact_out_top_slow", "qname", "Top QNAMES in transactions where host is the client and transaction speed is slower than p90",
               tops_of(b, TM_SLOW_OUT), topn, pct);
    }
    if (g & PV_DNS_TOP_PORTS)
        p.topn("dns_top_udp_ports", "port", "Top UDP source port on the query side of a transaction", dense_tops(&b.sum[PV_OFF_PORT], PV_PORT_BINS, 0), topn, pct);
    if (g & PV_DNS_TOP_ECS) {
        if (g & PV_DNS_COUNTERS) p.gauge("dns_wire_packets_query_ecs", "Total queries that have EDNS Client Subnet (ECS) field set", d[DC_QECS]);
        // geo / ASN of the subnet: no MaxMind database, those TopNs write nothing
        p.topn("dns_top_query_ecs", "ecs", "Top EDNS Client Subnet (ECS) observed in DNS queries", tops_of(b, TM_ECS), topn, pct);
    }
    if (g & PV_DNS_TOP_QNAMES) {
        p.topn("dns_top_qname2", "qname", "Top QNAMES, aggregated at a depth of two labels", tops_of(b, TM_QNAME2), topn, pct);
        p.topn("dns_top_qname3", "qname", "Top QNAMES, aggregated at a depth of three labels", tops_of(b, TM_QNAME3), topn, pct);
        p.topn("dns_top_nxdomain", "qname", "Top QNAMES with result code NXDOMAIN", tops_of(b, TM_NX), topn, pct);
        p.topn("dns_top_refused", "qname", "Top QNAMES with result code REFUSED", tops_of(b, TM_REFUSED), topn, pct);
        p.topn("dns_top_srvfail", "qname", "Top QNAMES with result code SRVFAIL", tops_of(b, TM_SRVFAIL), topn, pct);
        p.topn("dns_top_nodata", "qname", "Top QNAMES with result code NOERROR and no answer section", tops_of(b, TM_NODATA), topn, pct);
        if (g & PV_DNS_TOP_QNAMES_DETAILS) {
            p.topn("dns_top_qname_by_resp_bytes", "qname", "Top QNAMES by response volume in bytes", tops_of(b, TM_SIZED), topn, pct);
            p.topn("dns_top_noerror", "qname", "Top QNAMES with result code NOERROR", tops_of(b, TM_NOERROR), topn, pct);
        }
    }
    p.topn("dns_top_rcode", "rcode", "Top result codes", dense_tops(&b.sum[PV_OFF_RCODE], PV_RCODE_BINS, 2), topn, pct);
    p.topn("dns_top_qtype", "qtype", "Top query types", dense_tops(&b.sum[PV_OFF_QTYPE], PV_QTYPE_BINS, 1), topn, pct);
}

// NetworkMetricsBucket::to_prometheus / to_opentelemetry, Net v2
// (src/handlers/net/v2/NetStreamHandler.cpp:333-383; names NetStreamHandler.h:72-181): the
// event counts, `filtered_packets`, then per direction the bucket has seen, labelled
// direction=in|out|unknown (rates are timer-driven and out of scope; geo / ASN TopNs empty)
template <class Sink>
void net2_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET2];
    const uint32_t g = c->net2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    p.gauge("net_observed_packets", "Total packets events generated", n[N2_EVENTS]);
    p.gauge("net_deep_sampled_packets", "Total packets that were sampled for deep inspection", n[N2_SAMPLES]);
    if (g & PV_N2G_COUNTERS) p.gauge("net_filtered_packets", "Total packets seen that did not match the configured filter(s) (if any)", n[N2_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    const PromLabels base = p.add;
    for (uint32_t d = 0; d < 3; d++) {
        const uint64_t *dc = n + N2_DIR + 8 * d;
        if (!dc[N2_TOTAL]) continue;
        p.add = base;
        p.add["direction"] = dirs[d];
        if (g & PV_N2G_COUNTERS) {
            p.gauge("net_udp_packets", "Count of UDP packets", dc[N2_UDP]);
            p.gauge("net_tcp_packets", "Count of TCP packets", dc[N2_TCP]);
            p.gauge("net_other_l4_packets", "Count of packets which are not UDP or TCP", dc[N2_OTHER]);
            p.gauge("net_ipv4_packets", "Count of IPv4 packets", dc[N2_V4]);
            p.gauge("net_ipv6_packets", "Count of IPv6 packets", dc[N2_V6]);
            p.gauge("net_tcp_syn_packets", "Count of TCP SYN packets", dc[N2_SYN]);
            p.gauge("net_total_packets", "Count of total packets matching the configured filter(s)", dc[N2_TOTAL]);
        }
        if (g & PV_N2G_CARDINALITY)
            p.gauge("net_cardinality_ips", "IP cardinality", lround(cpc_estimate(&b.cpc[(CPC_V2 + d) * PV_CPC_COUPONS], b.merged)));
        if (g & PV_N2G_TOP_IPS) {
            p.topn("net_top_ipv4_packets", "ipv4", "Top IPv4 addresses", tops_of(b, TMH_V2_IP4 + d), topn, pct);
            p.topn("net_top_ipv6_packets", "ipv6", "Top IPv6 addresses", tops_of(b, TMH_V2_IP6 + d), topn, pct);
        }
        if (g & PV_N2G_QUANTILES) {
            uint64_t cnt;
            const uint64_t *h = &b.sum[PV_OFF_PAYLOAD2 + d * PV_PAYLOAD_BINS];
            auto q = hist_quantiles(h, PV_PAYLOAD_BINS, cnt);
            if (cnt && !b.qs_payload2[d].empty()) q = b.qs_payload2[d];
            uint64_t mx = 0;
            for (size_t i = 0; i < PV_PAYLOAD_BINS; i++)
                if (h[i]) mx = i;
            if (cnt) p.template summary<uint64_t>("net_payload_size_bytes", "Quantiles of payload sizes, in bytes", q, mx, cnt);
        }
    }
    p.add = base;
}

// DnsMetricsBucket::to_prometheus / to_opentelemetry, DNS v2
// (src/handlers/dns/v2/DnsStreamHandler.cpp:759-842; names DnsStreamHandler.h:98-115,250-270):
// the event counts, `filtered_packets`, then per transaction direction the bucket has set up
template <class Sink>
void dns2_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    const uint32_t g = c->dns2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    p.gauge("dns_observed_packets", "Total DNS wire packets events", d[DC_EVENTS]);
    p.gauge("dns_deep_sampled_packets", "Total DNS wire packets that were sampled for deep inspection", d[DC_SAMPLES]);
    if (g & PV_DNS2_COUNTERS)
        p.gauge("dns_filtered_packets", "Total DNS wire packets seen that did not match the configured filter(s) (if any)", d[DC_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    auto vmax = [](const auto &v) { return v.empty() ? 0 : *std::max_element(v.begin(), v.end()); };
    const PromLabels base = p.add;
    for (uint32_t x = 0; x < 3; x++) {
        const uint64_t *c2 = &b.sum[PV_OFF_DNS2 + x * PV_DNS2_CTRS];
        if (!c2[D2_SEEN]) continue;
        auto tops = [&](uint32_t metric) { return tops_of(b, TMH_V2_DNS + 4 * metric + x); };
        p.add = base;
        p.add["direction"] = dirs[x];
        if (g & PV_DNS2_COUNTERS) {
            p.gauge("dns_xacts", "Total DNS transactions (query/reply pairs)", c2[D2_XACTS]);
            p.gauge("dns_udp_xacts", "Total DNS transactions (query/reply pairs) received over UDP", c2[D2_UDP]);
            p.gauge("dns_tcp_xacts", "Total DNS transactions (query/reply pairs) received over TCP", c2[D2_TCP]);
            p.gauge("dns_dot_xacts", "Total DNS transactions (query/reply pairs) received over DNS over TLS", c2[D2_DOT]);
            p.gauge("dns_doh_xacts", "Total DNS transactions (query/reply pairs) received over DNS over HTTPS", c2[D2_DOH]);
            p.gauge("dns_dnscrypt_udp_xacts", "Total DNS transactions (query/reply pairs) received over DNSCrypt over UDP", c2[D2_CRYPT_UDP]);
            p.gauge("dns_dnscrypt_tcp_xacts", "Total DNS transactions (query/reply pairs) received over DNSCrypt over TCP", c2[D2_CRYPT_TCP]);
            p.gauge("dns_doq_xacts", "Total DNS transactions (query/reply pairs) received over DNS over QUIC", c2[D2_DOQ]);
            p.gauge("dns_ipv4_xacts", "Total DNS transactions (query/reply pairs) received over IPv4", c2[D2_V4]);
            p.gauge("dns_ipv6_xacts", "Total DNS transactions (query/reply pairs) received over IPv6", c2[D2_V6]);
            p.gauge("dns_nxdomain_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code NXDOMAIN", c2[D2_NX]);
            p.gauge("dns_ecs_xacts", "Total DNS transactions (query/reply pairs) with the EDNS Client Subnet option set", c2[D2_ECS]);
            p.gauge("dns_refused_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code REFUSED", c2[D2_REFUSED]);
            p.gauge("dns_srvfail_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code SRVFAIL", c2[D2_SRVFAIL]);
            p.gauge("dns_noerror_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code NOERROR", c2[D2_NOERROR]);
            p.gauge("dns_nodata_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code NOERROR but with an empty answers section", c2[D2_NODATA]);
            p.gauge("dns_authenticated_data_xacts", "Total DNS transactions (query/reply pairs) with the AD flag set in the response", c2[D2_AD]);
            p.gauge("dns_authoritative_answer_xacts", "Total DNS transactions (query/reply pairs) with the AA flag set in the response", c2[D2_AA]);
            p.gauge("dns_checking_disabled_xacts", "Total DNS transactions (query/reply pairs) with the CD flag set in the query", c2[D2_CD]);
            p.gauge("dns_timeout_queries", "Total number of DNS queries that timed out", c2[D2_TIMEOUT]);
            p.gauge("dns_orphan_responses", "Total number of DNS responses that do not have a corresponding query", c2[D2_ORPHAN]);
        }
        if (g & PV_DNS2_CARDINALITY)
            p.gauge("dns_cardinality_qname", "Cardinality of unique QNAMES, both ingress and egress",
                    lround(cpc_estimate(&b.cpc[(CPC_QNAME2 + x) * PV_CPC_COUPONS], b.merged)));
        if (g & PV_DNS2_TOP_PORTS)
            p.topn("dns_top_udp_ports_xacts", "port", "Top UDP source port on the query side of a transaction",
                   dense_tops(&b.sum[PV_OFF_PORT2 + x * PV_PORT_BINS], PV_PORT_BINS, 0), topn, pct);
        if (g & PV_DNS2_TOP_ECS)
            // geo / ASN of the subnet: no MaxMind database, those TopNs write nothing
            p.topn("dns_top_ecs_xacts", "ecs", "Top EDNS Client Subnet (ECS) observed in DNS transaction", tops(TM_ECS), topn, pct);
        if (g & PV_DNS2_TOP_RCODES) {
            p.topn("dns_top_nxdomain_xacts", "qname", "Top QNAMES with result code NXDOMAIN", tops(TM_NX), topn, pct);
            p.topn("dns_top_refused_xacts", "qname", "Top QNAMES with result code REFUSED", tops(TM_REFUSED), topn, pct);
            p.topn("dns_top_srvfail_xacts", "qname", "Top QNAMES with result code SRVFAIL", tops(TM_SRVFAIL), topn, pct);
            p.topn("dns_top_nodata_xacts", "qname", "Top QNAMES with result code NOERROR and empty answer section", tops(TM_NODATA), topn, pct);
            p.topn("dns_top_noerror_xacts", "qname", "Top QNAMES with result code NOERROR", tops(TM_NOERROR), topn, pct);
            p.topn("dns_top_rcode_xacts", "rcode", "Top result codes", dense_tops(&b.sum[PV_OFF_RCODE2 + x * PV_RCODE_BINS], PV_RCODE_BINS, 2),
                   topn, pct);
        }
        if (g & PV_DNS2_TOP_QNAMES) {
            p.topn("dns_top_qname2_xacts", "qname", "Top QNAMES, aggregated at a depth of two labels", tops(TM_QNAME2), topn, pct);
            p.topn("dns_top_qname3_xacts", "qname", "Top QNAMES, aggregated at a depth of three labels", tops(TM_QNAME3), topn, pct);
        }
        if (g & PV_DNS2_TOP_SIZE) {
            p.topn("dns_top_response_bytes", "qname", "Top QNAMES by response volume in bytes", tops(TM_SIZED), topn, pct);
            const auto &r = b.ratio2[x];
            if (!r.empty())
                p.template summary<double>("dns_response_query_size_ratio", "Quantiles of ratio of packet sizes in a DNS transaction (reply/query)",
                                           b.qs_ratio2[x].empty() ? quantiles(r) : b.qs_ratio2[x], vmax(r), r.size());
        }
        if (g & PV_DNS2_TOP_QTYPES)
            p.topn("dns_top_qtype_xacts", "qtype", "Top query types", dense_tops(&b.sum[PV_OFF_QTYPE2 + x * PV_QTYPE_BINS], PV_QTYPE_BINS, 1),
                   topn, pct);
        if (g & PV_DNS2_XACT_TIMES) {
            const auto &t = b.time2[x];
            if (!t.empty())
                p.template summary<uint64_t>("dns_xact_time_us", "Quantiles of transaction timing (query/reply pairs) in microseconds",
                                             b.qs_time2[x].empty() ? quantiles(t) : b.qs_time2[x], vmax(t), t.size());
            p.histogram("dns_xact_histogram_us", "Histogram of transaction timing (query/reply pairs) in microseconds", b.hist_time2(x));
            p.topn("dns_top_slow_xacts", "qname", "Top QNAMES in transactions where host is the server and transaction speed is slower than p90",
                   tops(TM_SLOW_OUT), topn, pct);
        }
    }
    p.add = base;
}

// KLL inclusive rank rule on exact data
uint64_t quantile_at(std::vector<uint64_t> v, double r)
{
    // the element of rank ceil(r n) - 1 of the sorted values: a selection, not a sort (a period
    // shift's thresholds select over every transaction of the bucket that closed)
    uint64_t w = (uint64_t)std::ceil(r * (double)v.size());
    size_t idx = w == 0 ? 0 : (size_t)(w - 1);
    if (idx >= v.size()) idx = v.size() - 1;
    std::nth_element(v.begin(), v.begin() + idx, v.end());
    return v[idx];
}

// copy the transaction values appended on the device since the last sync
int sync_xvals(pv_ctx *c)
{
    flush_fills(c);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    uint32_t status[ST_WORDS], nv = 0;
    if (!hip_ok(e = hipMemcpy(status, c->d_status, sizeof status, hipMemcpyDeviceToHost)) ||
        !hip_ok(e = hipMemcpy(&nv, c->d_nvals, 4, hipMemcpyDeviceToHost)))
        return c->hipfail(e, "status");
    if (status[ST_FLAGS] & PVF_VALUES_FULL || nv > c->xv_cap)
        return c->fail(PV_ECAPACITY, "transaction value buffer full");
    if (nv > c->xvals_synced) {
        size_t old = c->xvals_host.size(), add = nv - c->xvals_synced;
        c->xvals_host.resize(old + add);
        if (!hip_ok(e = hipMemcpy(&c->xvals_host[old], c->d_xvals + c->xvals_synced, add * sizeof(PvXValue),
                                  hipMemcpyDeviceToHost)))
            return c->hipfail(e, "transaction values");
        c->xvals_synced = nv;
    }
    return 0;
}

int window_slots(pv_ctx *c, const Window &w, uint32_t period, bool merged, std::vector<uint32_t> &out)
{
    out.clear();
    if (!merged) {
        if (period >= c->cfg.num_periods)
            return c->fail(PV_EINVAL, "invalid metrics period, specify [0, %u]", c->cfg.num_periods - 1);
        if (period >= w.slots.size())
            return c->fail(PV_EINVAL, "requested metrics period has not yet accumulated, current range is [0, %zu]",
                           w.slots.size() - 1);
        out.push_back(w.slots[period]);
        return 0;
    }
    if (period <= 1 || period > c->cfg.num_periods)
        return c->fail(PV_EINVAL, "invalid metrics period, specify [2, %u]", c->cfg.num_periods);
    for (size_t i = 0; i < w.slots.size() && i < period; i++) out.push_back(w.slots[i]);
    return 0;
}

} // namespace

// the merge entry points rewrite the window with other shards' data (note at pv_ctx::merged)
static void mark_merged(pv_ctx *c, const char *by)
{
    if (!c) return;
    c->merged = true;
    if (!c->merged_by) c->merged_by = by;
}
static int merged_refuse(pv_ctx *c)
{
    if (!c->merged) return 0;
    return c->fail(PV_EINVAL, "the window was merged across ranks (%s): a merged window is read-only until pv_reset",
                   c->merged_by ? c->merged_by : "merge");
}

// ====================================================================== C ABI
extern "C" {

const char *pv_version(void) { return "pvgpu 0.1 (gfx950)"; }

int pv_device_count(int *count)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return 0;
}

const char *pv_last_error(const pv_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void pv_free(void *p) { free(p); }

int pv_dns_code(int kind, const char *name, uint32_t *value)
{
    if (!name || !value || (kind != 0 && kind != 1)) return PV_EINVAL;
    const auto &m = kind == 0 ? rcode_names() : qtype_names();
    std::string n(name);
    if (n.empty()) return PV_EINVAL;
    if (std::all_of(n.begin(), n.end(), [](unsigned char ch) { return std::isdigit(ch); })) {
        if (n.size() > 6) return PV_EINVAL;
        const unsigned long v = std::stoul(n);
        if (!m.count((uint16_t)v) || v > 65535) return PV_EINVAL;
        *value = (uint32_t)v;
        return 0;
    }
    std::transform(n.begin(), n.end(), n.begin(), [](unsigned char ch) { return (char)std::toupper(ch); });
    for (const auto &kv : m)
        if (n == kv.second) { *value = kv.first; return 0; }
    return PV_EINVAL;
}

int pv_set_tcp_reassembly_limit(pv_ctx *c, uint64_t limit)
{
    if (!c) return PV_EINVAL;
    if (c->records_seen) return c->fail(PV_EINVAL, "tcp_packet_reassembly_cache_limit must be set before the first batch");
    c->tcp_limit = limit;
    return 0;
}

int pv_set_tcp_exact_lru(pv_ctx *c, int on)
{
    if (!c) return PV_EINVAL;
    if (c->records_seen) return c->fail(PV_EINVAL, "the exact TCP LRU mode must be set before the first batch");
    c->tcp_exact = on != 0;
    return 0;
}

// the public_suffix_list table on the device and the per-record suffix sizes (v1 and v2)
static int psl_setup(pv_ctx *c)
{
    hipError_t e = hipSuccess;
    if (!c->d_psl) {
        const std::vector<uint32_t> blob = pvname::psl_blob();
        if (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_psl, blob.size() * 4)) ||
            !hip_ok(e = hipMemcpy(c->d_psl, blob.data(), blob.size() * 4, hipMemcpyHostToDevice)))
            return c->hipfail(e, "public_suffix_list table");
    }
    if (!c->d_sfx && (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_sfx, c->max_records + 64))))
        return c->hipfail(e, "public_suffix_list record buffer");
    return 0;
}

int pv_set_dns_filters(pv_ctx *c, const pv_dns_filters *f)
{
    if (!c) return PV_EINVAL;
    if (c->records_seen) return c->fail(PV_EINVAL, "DNS filters must be set before the first batch");
    if (!f) { c->f_flags = c->f_rcode_mask = c->f_ancount = c->f_nq = c->f_nqn = c->f_nsx = 0; return 0; }
    uint32_t fl = 0;
    if (f->v2) {
        // DnsStreamHandler v2 start (dns/v2/DnsStreamHandler.cpp:61-170): one rcode mask for
        // exclude_noerror (every rcode but NOERROR) or only_rcode, tested on responses only
        if (!c->dns2_groups) return c->fail(PV_EINVAL, "v2 DNS filters without the DNS v2 handler");
        if (f->only_queries || f->only_responses || f->filter_all)
            return c->fail(PV_EUNSUPPORTED, "only_queries / only_responses / geo filters are not DNS v2 filters here");
        fl |= PVDF_V2;
        uint32_t mask = 0;
        if (f->exclude_noerror) mask = 0xfffeu;
        else if (f->only_rcode_mask) {
            for (uint32_t r = 0; r < 32; r++)
                if ((f->only_rcode_mask >> r) & 1 && (r > 15 || !rcode_names().count((uint16_t)r)))
                    return c->fail(PV_EINVAL, "DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode");
            mask = f->only_rcode_mask;
        }
        if (mask) fl |= PVDF2_RCODE;
        if (f->answer_count >= 0) fl |= PVDF_ANSWER_COUNT;
        if (f->only_dnssec_response) fl |= PVDF_ONLY_DNSSEC;
        if (f->xact_dirs_disabled & 1) fl |= PVDF2_NOIN;
        if (f->xact_dirs_disabled & 2) fl |= PVDF2_NOOUT;
        if (f->xact_dirs_disabled & 4) fl |= PVDF2_NOUNK;
        if (f->n_qtypes > PV_MAX_QTYPES) return c->fail(PV_EINVAL, "only_qtype: at most %d qtypes", PV_MAX_QTYPES);
        for (uint32_t k = 0; k < f->n_qtypes; k++)
            if (!qtype_names().count(f->qtypes[k]))
                return c->fail(PV_EINVAL, "DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: %u",
                               (unsigned)f->qtypes[k]);
        if (f->n_qtypes) fl |= PVDF_ONLY_QTYPE;
        if (f->n_qnames > PV_MAX_QNAMES) return c->fail(PV_EINVAL, "only_qname: at most %d names", PV_MAX_QNAMES);
        for (uint32_t k = 0; k < f->n_qnames; k++) {
            const char *q = f->qnames ? f->qnames[k] : nullptr;
            if (!q || !*q || strlen(q) > 255) return c->fail(PV_EINVAL, "only_qname: empty or over-long name");
            c->f_qn[k] = pvname::name_fp(q, strlen(q));
        }
        c->f_nqn = f->n_qnames;
        if (f->n_qnames) fl |= PVDF2_QNAME;
        if (f->n_qname_suffixes > PV_MAX_SUFFIXES)
            return c->fail(PV_EINVAL, "only_qname_suffix: at most %d suffixes", PV_MAX_SUFFIXES);
        for (uint32_t k = 0; k < f->n_qname_suffixes; k++) {
            const char *q = f->qname_suffixes ? f->qname_suffixes[k] : nullptr;
            if (!q || strlen(q) > 254) return c->fail(PV_EINVAL, "only_qname_suffix: missing or over-long suffix");
            c->f_sxl[k] = (uint32_t)strlen(q);
            c->f_sxh[k] = pvname::name_ph(q, strlen(q));
        }
        c->f_nsx = f->n_qname_suffixes;
        if (f->n_qname_suffixes) {
            fl |= PVDF_ONLY_QSUFFIX;
            hipError_t e;
            if (!c->d_sfx && (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_sfx, c->max_records + 64))))
                return c->hipfail(e, "only_qname_suffix record buffer");
        }
        // public_suffix_list (_configs, dns/v2/DnsStreamHandler.cpp:192-194,612-619): only while
        // only_qname_suffix is off; a response's own size aggregates its transaction's names
        if (f->public_suffix_list && !f->n_qname_suffixes) {
            if (int rc = psl_setup(c)) return rc;
            fl |= PVDF_PSL;
        }
        c->f_flags = fl;
        c->f_rcode_mask = mask;
        c->f_ancount = f->answer_count >= 0 ? (uint32_t)f->answer_count : 0;
        c->f_nq = f->n_qtypes;
        for (uint32_t k = 0; k < f->n_qtypes; k++) c->f_qt[k] = f->qtypes[k];
        return 0;
    }
    if (f->exclude_noerror) fl |= PVDF_EXCLUDE_NOERROR;
    else if (f->only_rcode_mask) {
        for (uint32_t r = 0; r < 32; r++)
            if ((f->only_rcode_mask >> r) & 1 && (r > 15 || !rcode_names().count((uint16_t)r)))
                // a DNS header carries a 4-bit rcode: extended rcodes can never match
                return c->fail(PV_EINVAL, "DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode");
        fl |= PVDF_ONLY_RCODE;
    }
    if (f->answer_count >= 0) fl |= PVDF_ANSWER_COUNT;
    if (f->only_queries) fl |= PVDF_ONLY_QUERIES;
    if (f->only_responses) fl |= PVDF_ONLY_RESPONSES;
    if (f->only_dnssec_response) fl |= PVDF_ONLY_DNSSEC;
    if (f->filter_all) fl |= PVDF_FILTER_ALL;
    if (f->n_qtypes > PV_MAX_QTYPES) return c->fail(PV_EINVAL, "only_qtype: at most %d qtypes", PV_MAX_QTYPES);
    for (uint32_t k = 0; k < f->n_qtypes; k++)
        if (!qtype_names().count(f->qtypes[k]))
            return c->fail(PV_EINVAL, "DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: %u",
                           (unsigned)f->qtypes[k]);
    if (f->n_qtypes) fl |= PVDF_ONLY_QTYPE;
    if (f->n_qnames > PV_MAX_QNAMES) return c->fail(PV_EINVAL, "only_qname: at most %d names", PV_MAX_QNAMES);
    if (f->n_qnames && (fl & PVDF_ONLY_RCODE))
        return c->fail(PV_EINVAL, "only_qname and only_rcode both install an input predicate: use one");
    for (uint32_t k = 0; k < f->n_qnames; k++) {
        const char *q = f->qnames ? f->qnames[k] : nullptr;
        if (!q || !*q || strlen(q) > 255) return c->fail(PV_EINVAL, "only_qname: empty or over-long name");
        c->f_qn[k] = pvname::name_fp(q, strlen(q)); // NameStats lower-cases, as only_qname's qname_ci (:151-160)
    }
    c->f_nqn = f->n_qnames;
    if (f->n_qnames) fl |= PVDF_ONLY_QNAME;
    if (f->n_qname_suffixes > PV_MAX_SUFFIXES)
        return c->fail(PV_EINVAL, "only_qname_suffix: at most %d suffixes", PV_MAX_SUFFIXES);
    for (uint32_t k = 0; k < f->n_qname_suffixes; k++) {
        const char *q = f->qname_suffixes ? f->qname_suffixes[k] : nullptr;
        if (!q || strlen(q) > 254) return c->fail(PV_EINVAL, "only_qname_suffix: missing or over-long suffix");
        c->f_sxl[k] = (uint32_t)strlen(q);
        c->f_sxh[k] = pvname::name_ph(q, strlen(q));
    }
    c->f_nsx = f->n_qname_suffixes;
    // public_suffix_list (DnsStreamHandler::_configs, dns/v1/DnsStreamHandler.cpp:648-657,
    // v2 :612-619): a config, not a filter, and only while only_qname_suffix is off. v2 applies
    // the size of a response's own first query name to its transaction's top_qname2/3
    // (new_dns_transaction :1067-1072)
    if (f->public_suffix_list && !f->n_qname_suffixes) {
        if (int rc = psl_setup(c)) return rc;
        fl |= PVDF_PSL;
    }
    if (f->n_qname_suffixes) {
        fl |= PVDF_ONLY_QSUFFIX;
        hipError_t e;
        if (!c->d_sfx && (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_sfx, c->max_records + 64))))
            return c->hipfail(e, "only_qname_suffix record buffer");
    }
    c->f_flags = fl;
    c->f_rcode_mask = (fl & PVDF_ONLY_RCODE) ? f->only_rcode_mask : 0;
    c->f_ancount = f->answer_count >= 0 ? (uint32_t)f->answer_count : 0;
    c->f_nq = f->n_qtypes;
    for (uint32_t k = 0; k < f->n_qtypes; k++) c->f_qt[k] = f->qtypes[k];
    return 0;
}

int pv_create(const pv_config *cfg, pv_ctx **out)
{
    *out = nullptr;
    if (!cfg) return PV_EINVAL;
    pv_ctx *c = new pv_ctx();
    c->cfg = *cfg;
    if (c->cfg.num_periods == 0) c->cfg.num_periods = 5;
    c->cfg.num_periods = std::max(1u, std::min(c->cfg.num_periods, 10u));
    if (c->cfg.topn_count == 0) c->cfg.topn_count = 10;
    if (c->cfg.xact_ttl_ms == 0) c->cfg.xact_ttl_ms = 5000;
    if (c->cfg.linktype == 0) c->cfg.linktype = 1;
    // group bits, 0 = the handler's defaults; PV_GROUPS_SET marks an explicit set (which may be empty)
    if (c->cfg.net_groups) c->net_groups = c->cfg.net_groups & ~PV_GROUPS_SET;
    if (c->cfg.dns_groups) c->dns_groups = c->cfg.dns_groups & ~PV_GROUPS_SET;
    if (c->cfg.net2_groups)
        c->net2_groups = PV_N2G_ON | ((c->cfg.net2_groups & PV_GROUPS_SET) ? (c->cfg.net2_groups & PV_NET2_DEFAULT_GROUPS)
                                                                           : PV_NET2_DEFAULT_GROUPS);
    if (c->cfg.dns2_groups) {
        c->dns2_groups = PV_N2G_ON | ((c->cfg.dns2_groups & PV_GROUPS_SET) ? (c->cfg.dns2_groups & 0x3ffu)
                                                                           : PV_DNS2_DEFAULT_GROUPS);
        // v1's DNS pass runs for the events (and their counts) only
        c->dns_groups = PV_DNS_TRANSACTIONS;
    }
    if (c->cfg.table_log2) c->tcap_log2 = c->cfg.table_log2;
    if (c->tcap_log2 < 8 || c->tcap_log2 > PV_REGION_LOG2 + PV_MAX_REGIONS_LOG2) {
        *out = c;
        return c->fail(PV_EINVAL, "table_log2 %u out of range [8, %d]", c->tcap_log2, PV_REGION_LOG2 + PV_MAX_REGIONS_LOG2);
    }
    c->reg_log2 = c->tcap_log2 > PV_REGION_LOG2 ? c->tcap_log2 - PV_REGION_LOG2 : 0;
    c->nn_cap = (uint32_t)std::min<uint64_t>(1ull << c->tcap_log2, 1ull << 22);
    if (c->cfg.max_records == 0) c->cfg.max_records = 1 << 20;
    c->max_records = c->cfg.max_records;
    c->ovf_cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(2 * c->max_records, 1u << 16), 1ull << 28);
    // deep_sample_rate (AbstractMetricsManager::configure, src/AbstractMetricsManager.h:357-365: > 100 -> 100, < 1 -> 1)
    c->sample_rate = c->cfg.deep_sample_rate == 0 ? 100u : std::max(1u, std::min(c->cfg.deep_sample_rate, 100u));
    if (c->sample_rate < 100 && c->cfg.net_filter_all) {
        *out = c;
        return c->fail(PV_EUNSUPPORTED, "deep_sample_rate below 100 with geo filters is not built");
    }
    // TransactionManager(ttl_ms) split (TransactionManager.h:60-68)
    if (c->cfg.xact_ttl_ms > 1000) { c->ttl_s = c->cfg.xact_ttl_ms / 1000; c->ttl_ms = c->cfg.xact_ttl_ms - c->ttl_s * 1000; }
    else c->ttl_ms = c->cfg.xact_ttl_ms;
    int rc = parse_host_spec(c, cfg->host_spec);
    if (rc) { *out = c; return rc; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { *out = c; return c->fail(PV_ENODEV, "no HIP device"); }
    if (cfg->device >= 0) {
        if (cfg->device >= ndev) { *out = c; return c->fail(PV_EINVAL, "device %d out of range", cfg->device); }
        c->device = cfg->device;
    } else {
        hipGetDevice(&c->device);
    }
    hipSetDevice(c->device);
    hipError_t e;
    uint64_t tcap = 1ull << c->tcap_log2;
    uint64_t mr = c->max_records;
    hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
    {
        // the grid's partition of a batch (DNS pass, combine, merge and the general Net passes):
        // three workgroups per CU; the register-window Net pass walks it with one workgroup per
        // CU (reg_wg_per_cu). PV_NET_WGCU / PV_REG_WGCU override them for A/B runs
        c->wg_per_cu = 3;
        if (const char *w = getenv("PV_NET_WGCU")) { c->wg_per_cu = std::max(1, atoi(w)); c->wg_forced = true; }
        if (const char *w = getenv("PV_REG_WGCU")) c->reg_wg_per_cu = std::max(1, atoi(w));
        {
            int nb = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(pv_dns_kernel), 64 * PV_DNS_WAVES, 0) == hipSuccess &&
                nb > 0)
                c->dns_wg_per_cu = nb;
        }
        if (const char *w = getenv("PV_DNS_WGCU")) c->dns_wg_per_cu = std::max(1, atoi(w));
    }
    // event / DNS work-list regions: main workgroups own wt_per_block * 64 slots each (the
    // last may overhang the batch by < wt_per_block tiles), boundary workgroups 64 each
    // (the last workgroup's region may overhang the batch by < wt_per_block tiles)
    // DNS over TCP messages of one batch (pv_dns_tcp appends their events behind the UDP
    // regions: one more region of slack)
    c->tmsg_cap = (uint32_t)std::min<uint64_t>(mr + 65536, 0x7fffffffull);
    c->tseg_cap = (uint32_t)std::min<uint64_t>(mr + 64, 0xffffffffull);
    const uint64_t region_max = mr / ((uint64_t)c->wg_per_cu * c->cus) + 64 * 64;
    const uint64_t ev_cap = mr + region_max + 64 * 64 + 16 * 256 + c->tmsg_cap + 2 * region_max;
    c->pend_cap = 2 * mr; // open queries carried between batches
    c->ev_store_cap = std::max<uint64_t>(ev_cap, c->pend_cap + mr);
    c->key_cap = mr + c->tmsg_cap + c->pend_cap;
    const size_t esc = (size_t)c->ev_store_cap, kc = (size_t)c->key_cap;
    c->orph_cap = (uint32_t)std::min<uint64_t>(2 * mr, 1u << 30);
    if (!hip_ok(e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) ||
        !hip_ok(e = hipMalloc(&c->d_sum, (size_t)PV_SLOTS * PV_SUM_WORDS * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_cpc, (size_t)PV_SLOTS * PV_MIN_WORDS * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tkeys, (size_t)PV_TABLES * tcap * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tcnt, (size_t)PV_TABLES * tcap * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_taux, (size_t)PV_TABLES * tcap * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_arena, (size_t)PV_TABLES * c->arena_cap)) ||
        !hip_ok(e = hipMalloc(&c->d_arena_top, PV_TABLES * PV_ARENA_PARTS * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_dbits, (size_t)(mr / 64 + 2) * 8)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_dbits, (size_t)(mr / 64 + 2) * 8, hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_events, esc * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_ekeys, (size_t)ev_cap * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_mq_cnt, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_dq, (size_t)ev_cap * 32)) ||
        !hip_ok(e = hipMalloc(&c->d_dq_cnt, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_stamps, 65536 * 4 * 8 * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_blk_events, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_orph, (size_t)c->orph_cap * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_pend[0], esc * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_pend[1], esc * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_pkeys[0], kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_pkeys[1], kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_pvals[0], kc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_pvals[1], kc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_skeys, kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_skeys2, kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_svals, kc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_svals2, kc * 4)) ||
        !hip_ok(e = (c->xv_cap = (uint64_t)mr * 2, hipMalloc(&c->d_xvals, (size_t)mr * 2 * sizeof(PvXValue)))) ||
        !hip_ok(e = hipMalloc(&c->d_valid, (size_t)mr * sizeof(PvXValid))) ||
        !hip_ok(e = hipMalloc(&c->d_nvals, 16)) ||
        // one read-back block: the status words, the tables' live counts, the two overflow
        // words (a batch reads them back with one copy)
        !hip_ok(e = hipMalloc(&c->d_status, ST_RB_WORDS * 4)) ||
        !hip_ok(e = (c->d_tab_live = c->d_status + ST_ALLOC, c->d_ovf_cnt = c->d_tab_live + PV_TABLES, hipSuccess)) ||
        !hip_ok(e = hipMemsetAsync(c->d_status, 0, ST_RB_WORDS * 4, c->stream)) ||
        !hip_ok(e = hipMalloc(&c->d_theta, ((size_t)1 << c->reg_log2) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_ovf, (size_t)c->ovf_cap * sizeof(PvOvf))) ||
        ((c->dns2_groups & PV_DNS2_TOP_ECS) &&
         (!hip_ok(e = hipMalloc(&c->d_eecs, esc * 8)) ||
          !hip_ok(e = hipMalloc(&c->d_pecs[0], esc * 8)) ||
          !hip_ok(e = hipMalloc(&c->d_pecs[1], esc * 8)))) ||
        !hip_ok(e = hipMalloc(&c->d_ovf2, (size_t)c->ovf_cap * sizeof(PvOvf))) ||

        !hip_ok(e = hipMalloc(&c->d_nn, (size_t)c->nn_cap * sizeof(PvNewName))) ||
        !hip_ok(e = hipMalloc(&c->d_iplog, (size_t)(mr + 64) * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_iplog32, (size_t)(mr + 64) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_ipx_rep, (size_t)(mr + 64) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_ipdir, (size_t)(mr / 64 + 2) * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_ipx_cnt, (size_t)PV_MAX_GRID * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_trash, (size_t)PV_TRASH_WAVES * 2048)) ||
        !hip_ok(e = hipMalloc(&c->d_cb_cnt, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_params, 2 * sizeof(PvParams))) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_params, 2 * sizeof(PvParams), hipHostMallocDefault)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_xparams, sizeof(PvXactParams), hipHostMallocDefault)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_status, ST_RB_WORDS * 4, hipHostMallocDefault)) ||
        !hip_ok(e = (c->h_tab_live = c->h_status + ST_ALLOC, c->h_ovf = c->h_tab_live + PV_TABLES, hipSuccess)) ||
        !hip_ok(e = hipMalloc(&c->d_tseg, (size_t)c->tseg_cap * sizeof(PvTcpSeg))) ||
        !hip_ok(e = hipMalloc(&c->d_tmask, (size_t)(mr / 64 + 2) * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tpm, (size_t)(mr / 64 + 2) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_tcpcnt, (PVT_WORDS + 1) * 4)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_tcpcnt, (PVT_WORDS + 1) * 4, hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_tparams, sizeof(PvTcpParams))) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_tparams, sizeof(PvTcpParams), hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_xparams, sizeof(PvXactParams))) || !hip_ok(e = hipEventCreate(&c->ev_start)) ||
        !hip_ok(e = hipEventCreate(&c->ev_stop))) {
        *out = c;
        return c->hipfail(e, "device allocation");
    }
    size_t tmp = 0;
    pv_radix_sort_pairs(nullptr, &tmp, c->d_skeys, c->d_skeys2, c->d_svals, c->d_svals2, kc, c->stream);
    c->sort_tmp_bytes = std::max<size_t>(tmp, 256);
    if (!hip_ok(e = hipMalloc(&c->d_sort_tmp, c->sort_tmp_bytes))) { *out = c; return c->hipfail(e, "sort scratch"); }
    *out = c;
    return pv_reset(c);
}

void pv_destroy(pv_ctx *c)
{
    if (c && c->hprof_on)
        fprintf(stderr, "pv_hostprof ms: wait=%.1f index=%.1f cut=%.1f shifts=%.1f kernels=%.1f tcp=%.1f pairs=%.1f tail=%.1f sync=%.1f loop=%.1f | launch=%.1f pend_in=%.1f sort=%.1f resolve=%.1f nv_sync=%.1f | X=%.1f memset=%.1f upload=%.1f launch=%.1f xsync=%.1f\n",
                c->hprof[0], c->hprof[1], c->hprof[2], c->hprof[3], c->hprof[4], c->hprof[5], c->hprof[6], c->hprof[7],
                c->hprof[8], c->hprof[9], c->hprof[14], c->hprof[10], c->hprof[11], c->hprof[12], c->hprof[13], c->hprof[15], c->hprof[16], c->hprof[17], c->hprof[18], c->hprof[19]);
    if (!c) return;
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    if (c->stream) { hipSetDevice(c->device); hipStreamSynchronize(c->stream); }
    void *ptrs[] = {c->d_sum, c->d_cpc, c->d_tkeys, c->d_tcnt, c->d_taux, c->d_arena, c->d_arena_top, c->d_events,
                    c->d_xvh, c->d_skeys, c->d_skeys2, c->d_svals, c->d_svals2, c->d_sort_tmp, c->d_xvals, c->d_status,
                    c->d_valid, c->d_nvals, c->d_params, c->d_xparams, c->d_ekeys, c->d_blk_events, c->d_mq, c->d_tpbuf, c->d_cb, c->d_cb_cnt, c->d_cb_h, c->d_nn, c->d_iplog, c->d_trash, c->d_mq_cnt, c->d_stamps, c->d_dq, c->d_dq_cnt,
                    c->stage[0].d_recs, c->stage[0].d_offs, c->stage[1].d_recs, c->stage[1].d_offs,
                    c->d_pend[0], c->d_pend[1], c->d_pkeys[0], c->d_pkeys[1], c->d_pvals[0], c->d_pvals[1], c->d_orph, c->d_orph_ord, c->d_sfx, c->d_psl,
                    c->d_tseg, c->d_tmask, c->d_tpm, c->d_tcpcnt, c->d_tparams, c->d_tkey[0], c->d_tkey[1], c->d_tval[0],
                    c->d_tval[1], c->d_run_flow, c->d_tsort_tmp, c->d_flows, c->d_carry[0], c->d_carry[1], c->d_clist[0],
                    c->d_clist[1], c->d_frags, c->d_marena, c->d_moffs, c->d_tmq, c->d_tsfx,
                    c->d_theta, c->d_ctmp, c->d_ctop, c->d_ovf, c->d_ovf2, c->d_iplog32,
                    c->d_ipx_rep, c->d_ipdir, c->d_ipx_cnt, c->d_slow, c->d_eecs, c->d_pecs[0], c->d_pecs[1], c->d_lru_ev, c->d_fclose,
                    c->d_xcnt, c->d_xrhdr, c->d_xtot, c->d_xsend, c->d_xrecv, c->d_xp, c->d_bpf, c->d_fwork, c->d_frecs,
                    c->d_foffs, c->d_fsc, c->d_fscan, c->d_eoc, c->d_eoc_cnt};
    for (void *p : ptrs) if (p) hipFree(p);
    if (c->d_dbits) hipFree(c->d_dbits);
    for (void *hp : {(void *)c->h_params, (void *)c->h_xparams, (void *)c->h_status, (void *)c->h_dbits, (void *)c->h_tcpcnt,
                     (void *)c->h_tparams})
        if (hp) hipHostFree(hp);
    for (auto &st : c->stage) {
        if (st.d_ix) hipFree(st.d_ix);
        if (st.h_ix) hipHostFree(st.h_ix);
        if (st.h_recs) hipHostFree(st.h_recs);
        if (st.h_offs) hipHostFree(st.h_offs);
        if (st.copied) hipEventDestroy(st.copied);
    }
    for (auto &r : c->ring) {
        if (r.d_buf) hipFree(r.d_buf);
        if (r.d_offs) hipFree(r.d_offs);
        if (r.h_stage) hipHostFree(r.h_stage);
        if (r.landed) hipEventDestroy(r.landed);
    }
    if (c->copy_stream) hipStreamDestroy(c->copy_stream);
    if (c->copy_stream2) hipStreamDestroy(c->copy_stream2);
    if (c->d_ndeep) hipFree(c->d_ndeep);
    if (c->h_ndeep) hipHostFree(c->h_ndeep);
    for (void *p : {(void *)c->d_fbits, (void *)c->d_tfbits, (void *)c->d_ntcp}) if (p) hipFree(p);
    for (void *p : {(void *)c->h_fbits, (void *)c->h_tfbits, (void *)c->h_ntcp}) if (p) hipHostFree(p);
    c->pool.reset();
    if (c->ev_start) hipEventDestroy(c->ev_start);
    if (c->ev_stop) hipEventDestroy(c->ev_stop);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

// TCP: no connection, no carried bytes, no TCP record seen
static void tcp_reset(pv_ctx *c)
{
    launch_fill32(c, c->d_tcpcnt + PVT_WORDS, 1, 0);
    if (c->d_flows) launch_fill32(c, (uint32_t *)c->d_flows, ((uint64_t)sizeof(PvTcpFlow) / 4) << c->flow_cap_log2, 0);
    c->n_clist = 0;
    c->carry_used = 0;
    c->tcp_active = false;
    c->lru.clear();
    c->lru_at.clear();
}

int pv_reset(pv_ctx *c)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    // device state stays as it is: which slot parts are clean carries over
    for (Window *w : {&c->net, &c->dns}) {
        bool cl[PV_SLOTS];
        memcpy(cl, w->clean, sizeof cl);
        *w = Window();
        memcpy(w->clean, cl, sizeof cl);
    }
    c->started = c->ended = false;
    c->records_seen = 0;
    c->draws_net.reset(Jsf32());
    c->draws_dns.reset(Jsf32());
    c->dns_deep_now = true;
    c->xvals_host.clear();
    c->xvals_synced = 0;
    c->from90 = c->to90 = 0.0f;
    c->p90_2[0] = c->p90_2[1] = c->p90_2[2] = 0.0f;
    c->remote_topn.clear();
    c->x_ranks = c->x_rank = 0;
    c->x_view_on = false;
    c->merged = false;
    c->merged_by = nullptr;
    c->x_view.clear();
    c->xq_on = false;
    c->xq.clear();
    c->n_pend = 0;
    c->pend_hi = 0;
    c->pend_base = -1;
    c->dns_shifts.clear();
    c->sg_ord.clear();
    c->sstore.clear();
    c->scands.clear();
    c->sorph.clear();
    c->orph_done = 0;
    c->xv_local_end = SIZE_MAX;
    c->slow_xv.clear();
    c->stubs.clear();
    c->edge_h = 0;
    c->dns_shift_ord.clear();
    launch_fill32(c, c->d_nvals, 4, 0); // with the next batch's slot clears
    tcp_reset(c);
    return 0;
}

int pv_set_global_base(pv_ctx *c, uint64_t base)
{
    c->global_base = base;
    return 0;
}

int pv_index_records(const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets, uint64_t max_records,
                     uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes, pv_index_info *info)
{
    (void)ts_nano;
    memset(info, 0, sizeof *info);
    info->monotone = 1;
    size_t pos = 0;
    uint64_t n = 0;
    uint32_t nc = 0;
    int64_t prev_sec = -1;
    while (pos + 16 <= bytes && n < max_records) {
        uint32_t h[4];
        memcpy(h, recs + pos, 16);
        if (pos + 16 + h[2] > bytes) break;
        if (pos > 0xffffffffull) return PV_EINVAL; // offsets are 32-bit: split larger runs
        offsets[n] = (uint32_t)pos;
        int64_t sec = h[0];
        int64_t nsec = ts_nano ? h[1] : (int64_t)h[1] * 1000;
        if (n == 0) { info->first_sec = sec; info->first_nsec = nsec; }
        info->last_sec = sec; info->last_nsec = nsec;
        if (sec != prev_sec) {
            if (sec < prev_sec) info->monotone = 0;
            if (nc < max_changes) { sc_idx[nc] = (uint32_t)n; sc_sec[nc] = (uint32_t)sec; }
            nc++;
            prev_sec = sec;
        }
        pos += 16 + h[2];
        n++;
    }
    info->n_records = n;
    info->bytes_used = pos;
    info->n_sec_changes = nc;
    if (nc > max_changes) return PV_ECAPACITY;
    return 0;
}

namespace {

// A period shift inside a batch: its threshold second (the shifting event's ts_sec) and the
// batch record index of that event (AbstractMetricsManager::new_event, src/AbstractMetricsManager.h:318-333)
struct Shift {
    int64_t sec;
    uint64_t idx;
    uint64_t ord; // DNS shifts: position of the shifting event (record * 4, + sub for a TCP message)
};

// The Net manager's shifts: every packet is a Net event, so the first record with
// ts_sec >= next_shift shifts, then next_shift = its second + 60, repeatedly.
void net_shifts_of(int64_t T, const pv_index_info *info, const uint32_t *sc_idx, const uint32_t *sc_sec,
                   std::vector<Shift> &out)
{
    for (uint32_t k = 0; k < info->n_sec_changes; k++)
        if ((int64_t)sc_sec[k] >= T) {
            out.push_back({(int64_t)sc_sec[k], sc_idx[k], (uint64_t)sc_idx[k] * 4});
            T = (int64_t)sc_sec[k] + 60;
        }
}

uint64_t next_bit(const uint64_t *bits, uint64_t from, uint64_t n)
{
    for (uint64_t w = from >> 6; (w << 6) < n; w++) {
        uint64_t v = bits[w];
        if (w == (from >> 6)) v &= ~0ull << (from & 63);
        if (v) {
            const uint64_t i = (w << 6) + (uint64_t)__builtin_ctzll(v);
            return i < n ? i : n;
        }
    }
    return n;
}

// The DNS manager's shifts: the first DNS event (in stream order) with ts_sec >= next_shift, then
// next_shift = its second + 60, repeatedly (AbstractMetricsManager::new_event, per event: the
// batch's timestamps need not be monotone). DNS events: the UDP datagrams of pv_dns_prescan's
// bits, and the TCP messages (ord, stamp second) of the batch's TCP stage, whose stamps (a
// connection's end time) may lag their position.
void dns_shifts_of(int64_t T, const uint64_t *bits, uint64_t n, const pv_index_info *info, const uint32_t *sc_idx,
                   const uint32_t *sc_sec, const std::vector<std::pair<uint64_t, int64_t>> &tcp, std::vector<Shift> &out)
{
    const uint32_t nsc = info->n_sec_changes;
    uint32_t k = 0;     // the second-run holding record `after / 4`
    size_t t = 0;
    uint64_t after = 0; // events at ord >= after are still candidates
    for (;;) {
        // UDP: the first event at or past `after` whose record's second is >= T, run by run of
        // equal seconds (sc_idx / sc_sec: the batch's change points, in record order)
        const uint64_t from = (after + 3) / 4;
        while (k + 1 < nsc && sc_idx[k + 1] <= from) k++;
        uint64_t ui = n, uord = ~0ull;
        int64_t usec = 0;
        for (uint32_t kk = k; kk < nsc; kk++) {
            if ((int64_t)sc_sec[kk] < T) continue;
            const uint64_t lo = std::max<uint64_t>(sc_idx[kk], from), hi = kk + 1 < nsc ? sc_idx[kk + 1] : n;
            if (lo >= hi) continue;
            const uint64_t i = next_bit(bits, lo, hi);
            if (i < hi) {
                ui = i;
                usec = (int64_t)sc_sec[kk];
                uord = ui * 4;
                break;
            }
        }
        // TCP: the first message after the last shift whose stamp second is >= T
        while (t < tcp.size() && tcp[t].first < after) t++;
        size_t tt = t;
        while (tt < tcp.size() && tcp[tt].second < T && tcp[tt].first < uord) tt++;
        const bool tcp_first = tt < tcp.size() && tcp[tt].second >= T && tcp[tt].first < uord;
        if (tcp_first) {
            out.push_back({tcp[tt].second, tcp[tt].first / 4, tcp[tt].first});
            T = tcp[tt].second + 60;
            after = tcp[tt].first + 1;
            t = tt + 1;
            continue;
        }
        if (uord == ~0ull) return;
        out.push_back({usec, ui, uord});
        T = usec + 60;
        after = uord + 1;
    }
}

// parameter fields every kernel reads: record access, parse configuration, DNS filters
// A parameter block to device memory through pv_store_blob's kernel arguments (blocks up to
// 2 KiB; larger ones by copy)
static hipError_t upload_params(void *dst, const void *src, size_t bytes, hipStream_t st)
{
    if (bytes > sizeof(PvBlob) || ((uintptr_t)dst & 15)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    PvBlob b;
    memcpy(b.w, src, bytes);
    const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
    hipLaunchKernelGGL(pv_store_blob, dim3(1), dim3(PV_BLOB_WORDS), 0, st, b, (uint4 *)dst, n16);
    return hipGetLastError();
}

// The queued fills and a parameter block in one launch (pv_fill_store) when both fit; else the
// fills, then upload_params
static hipError_t fill_and_upload(pv_ctx *c, void *dst, const void *src, size_t bytes, hipStream_t st)
{
    static const char *nofuse = getenv("PV_FILL_FUSE"); // (=0: separate launches, A/B runs)
    if (!c->fills.n || st != c->stream || bytes > sizeof(PvBlob) || ((uintptr_t)dst & 15) || (nofuse && !strcmp(nofuse, "0"))) {
        flush_fills(c);
        return upload_params(dst, src, bytes, st);
    }
    PvBlob b;
    memcpy(b.w, src, bytes);
    const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
    hipSetDevice(c->device);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((c->fills_max + 255) / 256, 4096);
    static_assert(PV_BLOB_WORDS <= 256, "the blob's words in the first workgroup");
    hipLaunchKernelGGL(pv_fill_store, dim3(blocks), dim3(256), 0, c->stream, c->fills, b, (uint4 *)dst, n16);
    c->fills.n = 0;
    c->fills_max = 0;
    return hipGetLastError();
}

void params_common(pv_ctx *c, PvParams &P, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n)
{
    memset(&P, 0, sizeof P);
    P.recs = d_recs;
    P.offs = d_offs;
    P.n = n;
    P.linktype = c->cfg.linktype;
    P.ts_nano = c->cfg.ts_nano;
    P.net_groups = c->net_groups;
    P.dns_groups = c->dns_groups;
    P.net2_groups = c->net2_groups;
    P.dns2_groups = c->dns2_groups;
    P.net_filter_all = c->cfg.net_filter_all ? 1u : 0u;
    P.nets = c->nets;
    P.f_flags = c->f_flags;
    P.f_rcode_mask = c->f_rcode_mask;
    P.f_ancount = c->f_ancount;
    P.f_nq = c->f_nq;
    for (uint32_t k = 0; k < c->f_nq; k++) P.f_qt[k] = c->f_qt[k];
    P.f_nqn = c->f_nqn;
    for (uint32_t k = 0; k < c->f_nqn; k++) P.f_qn[k] = c->f_qn[k];
    P.f_nsx = c->f_nsx;
    P.sfx_of = c->d_sfx;
    P.psl = c->d_psl;
    for (uint32_t k = 0; k < c->f_nsx; k++) { P.f_sxl[k] = c->f_sxl[k]; P.f_sxh[k] = c->f_sxh[k]; }
    P.dbits = c->d_dbits;
    P.tseg = c->d_tseg;
    P.tseg_cap = c->tseg_cap;
    P.tseg_cnt = c->d_status + ST_TSEG;
    P.tmask = c->d_tmask;
}

// pv_dns_prescan over a batch, its bits copied to c->h_dbits (synchronises); with tcp_emit
// also the batch's TCP segments and tile masks (their counts into tseg[2])
int dns_prescan(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n, hipStream_t st, bool tcp_emit,
                uint32_t *tseg, bool fbits = false)
{
    launch_fill32(c, c->d_status + ST_TSEG, 2, 0);
    flush_fills(c);
    PvParams P;
    params_common(c, P, d_recs, d_offs, n);
    // 2: every TCP connection, 4: every TCP packet (the exact LRU mode: the LRU holds every
    // connection and runs its cleanup after every TCP packet)
    P.tcp_emit = tcp_emit ? (c->tcp_exact_on() ? 7u : 1u) : 0u;
    if (fbits) P.fbits = c->d_fbits;
    hipError_t e;
    *c->h_params = P;
    if (!hip_ok(e = upload_params(c->d_params, c->h_params, sizeof P, st)))
        return c->hipfail(e, "parameter upload");
    const uint64_t tiles = (n + 63) / 64;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((tiles + 3) / 4, (uint64_t)c->cus * 8);
    hipLaunchKernelGGL(pv_dns_prescan, dim3(grid), dim3(256), 0, st, (const PvParams *)c->d_params);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_dns_prescan");
    if (!hip_ok(e = hipMemcpyAsync(c->h_dbits, c->d_dbits, tiles * 8, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(c->h_status + ST_TSEG, c->d_status + ST_TSEG, 8, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "DNS prescan");
    tseg[0] = c->h_status[ST_TSEG];
    tseg[1] = c->h_status[ST_TSEG_BYTES];
    if (fbits && (!hip_ok(e = hipMemcpyAsync(c->h_fbits, c->d_fbits, tiles * 8, hipMemcpyDeviceToHost, st)) ||
                  !hip_ok(e = hipStreamSynchronize(st))))
        return c->hipfail(e, "DNS filter prescan");
    return 0;
}

// ---- DNS over TCP (pv_tcp.hip)
int grow_bytes(pv_ctx *c, void **p, uint64_t &cap, uint64_t need, size_t elem, const char *what)
{
    if (need <= cap && *p) return 0;
    if (*p) hipFree(*p);
    *p = nullptr;
    cap = 0;
    const uint64_t n = std::max<uint64_t>(need + need / 2, 1u << 16);
    hipError_t e;
    if (!hip_ok(e = hipMalloc(p, n * elem))) return c->hipfail(e, what);
    cap = n;
    return 0;
}
#define PV_GROW(c, p, cap, need, what) grow_bytes(c, (void **)&(p), cap, need, sizeof(*(p)), what)

// the stage's fixed buffers, on the first batch that holds a DNS-port TCP segment
int tcp_alloc(pv_ctx *c)
{
    if (c->tcp_alloced) return 0;
    hipError_t e;
    const uint64_t ns = c->tseg_cap, fc = 1ull << c->flow_cap_log2;
    if (!hip_ok(e = hipMalloc(&c->d_tkey[0], ns * 8)) || !hip_ok(e = hipMalloc(&c->d_tkey[1], ns * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tval[0], ns * 4)) || !hip_ok(e = hipMalloc(&c->d_tval[1], ns * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_run_flow, ns * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_flows, fc * sizeof(PvTcpFlow))) ||
        !hip_ok(e = hipMemsetAsync(c->d_flows, 0, fc * sizeof(PvTcpFlow), c->stream)) ||
        !hip_ok(e = hipMalloc(&c->d_clist[0], fc * 4)) || !hip_ok(e = hipMalloc(&c->d_clist[1], fc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_moffs, (size_t)c->tmsg_cap * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_tmq, (size_t)c->tmsg_cap * 32)) ||
        !hip_ok(e = hipMalloc(&c->d_tsfx, (size_t)c->tmsg_cap)))
        return c->hipfail(e, "TCP stage allocation");
    size_t tmp = 0;
    pv_tcp_sort(nullptr, &tmp, c->d_tkey[0], c->d_tkey[1], c->d_tval[0], c->d_tval[1], ns, c->stream);
    c->tsort_tmp_bytes = std::max<size_t>(tmp, 256);
    if (!hip_ok(e = hipMalloc(&c->d_tsort_tmp, c->tsort_tmp_bytes))) return c->hipfail(e, "TCP sort scratch");
    c->tcp_alloced = true;
    return 0;
}

// PcapInputStream's LRU list in the exact LRU mode (PcapInputStream.cpp:97-99,254-283,429-465),
// replayed over the batch's segments (every TCP packet) in capture order from the dry run's events
// (skey: sorted fkey << 32 | record index; sval: segment index per sorted key; ev per sorted key:
// flags | dir << 8, second, LRU time of the segment's last put). Per packet, as the reference: the
// reassembly's puts (a connection start with its start second, a message delivery with endTime,
// which is 0 until the connection's second packet) move the connection to the head and, past the
// limit, evict the tail; a FIN/RST close erases it; then at most MAX_TCP_CLEANUPS (100) connections
// leave from the tail while the tail's time + 30 s <= the packet's second, then the evicted ones
// close. Every connection closed this way is closed after that record (closeConnection): fclose
// (per segment index) at its first sorted segment when it has packets in the batch (its later
// packets are then Ignore_PacketOfClosedFlow, and their events are skipped here), else a
// close-only segment appended to `extra` with its fclose in `extra_fc`.
void tcp_lru_replay(pv_ctx *c, const std::vector<uint64_t> &skey, const std::vector<uint32_t> &sval,
                    const std::vector<uint32_t> &ev, std::vector<uint32_t> &fclose, std::vector<PvTcpSeg> &extra,
                    std::vector<uint32_t> &extra_fc)
{
    static constexpr int MAX_TCP_CLEANUPS = 100; // PcapInputStream.h:98
    const size_t n = skey.size();
    std::vector<uint32_t> order(n);
    std::unordered_map<uint32_t, uint32_t> first; // flow -> its first sorted segment
    for (size_t k = 0; k < n; k++) {
        order[k] = (uint32_t)k;
        if (!k || (skey[k] >> 32) != (skey[k - 1] >> 32)) first[(uint32_t)(skey[k] >> 32)] = (uint32_t)k;
    }
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return (uint32_t)skey[a] < (uint32_t)skey[b]; });
    auto erase = [&](uint32_t f) {
        auto it = c->lru_at.find(f);
        if (it == c->lru_at.end()) return;
        c->lru.erase(it->second);
        c->lru_at.erase(it);
    };
    std::unordered_map<uint32_t, bool> closed; // closed by the replay in this batch
    auto close_after = [&](uint32_t v, uint32_t idx, uint32_t sec, uint32_t dir) {
        erase(v);
        if (closed.count(v)) return;
        closed[v] = true;
        auto it = first.find(v);
        if (it != first.end()) {
            uint32_t *w = &fclose[3 * (size_t)sval[it->second]];
            w[0] = idx; w[1] = sec; w[2] = dir;
            return;
        }
        PvTcpSeg g;
        memset(&g, 0, sizeof g);
        g.idx = idx;
        g.fkey = v;
        g.sec = sec;
        g.flags = PV_TF_CLOSE;
        g.dirv6 = (uint8_t)dir;
        extra.push_back(g);
        extra_fc.insert(extra_fc.end(), {idx, sec, dir});
    };
    std::vector<uint32_t> overflow;
    auto put = [&](uint32_t f, uint32_t t) {
        erase(f);
        c->lru.emplace_front(f, t);
        c->lru_at[f] = c->lru.begin();
        if (c->tcp_limit && c->lru_at.size() > c->tcp_limit) {
            const uint32_t v = c->lru.back().first;
            c->lru_at.erase(v);
            c->lru.pop_back();
            overflow.push_back(v);
        }
    };
    for (uint32_t k : order) {
        const uint32_t f = (uint32_t)(skey[k] >> 32), idx = (uint32_t)skey[k];
        const uint32_t fl = ev[3 * k] & 0xff, dir = (ev[3 * k] >> 8) & 3, sec = ev[3 * k + 1], pt = ev[3 * k + 2];
        if (!closed.count(f)) {
            if (fl & PVT_EV_NEW) put(f, sec);
            if (fl & PVT_EV_PUT) put(f, pt);
            if (fl & PVT_EV_CLOSE) erase(f);
        }
        for (int q = 0; q < MAX_TCP_CLEANUPS && !c->lru.empty(); q++) {
            const auto back = c->lru.back();
            if ((uint64_t)sec < (uint64_t)back.second + PV_TCP_TIMEOUT) break;
            close_after(back.first, idx, sec, dir);
        }
        for (uint32_t v : overflow) close_after(v, idx, sec, dir);
        overflow.clear();
    }
}

// The segment arrays of the TCP stage for `need` segments (the end of a capture adds one per open
// connection to a batch's own), the first `keep` segments kept
int tcp_grow_segs(pv_ctx *c, uint64_t need, uint32_t keep, hipStream_t st)
{
    if (need <= c->tseg_cap) return 0;
    if (need > 0xffffffffull) return c->fail(PV_ECAPACITY, "TCP segments");
    hipError_t e;
    PvTcpSeg *seg = nullptr;
    if (!hip_ok(e = hipMalloc(&seg, need * sizeof(PvTcpSeg))) ||
        (keep && !hip_ok(e = hipMemcpyAsync(seg, c->d_tseg, (size_t)keep * sizeof(PvTcpSeg), hipMemcpyDeviceToDevice, st))) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "TCP segments");
    hipFree(c->d_tseg);
    c->d_tseg = seg;
    for (int k = 0; k < 2; k++) {
        hipFree(c->d_tkey[k]);
        hipFree(c->d_tval[k]);
        c->d_tkey[k] = nullptr;
        c->d_tval[k] = nullptr;
    }
    hipFree(c->d_run_flow);
    hipFree(c->d_tsort_tmp);
    c->d_run_flow = nullptr;
    c->d_tsort_tmp = nullptr;
    if (!hip_ok(e = hipMalloc(&c->d_tkey[0], need * 8)) || !hip_ok(e = hipMalloc(&c->d_tkey[1], need * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tval[0], need * 4)) || !hip_ok(e = hipMalloc(&c->d_tval[1], need * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_run_flow, need * 4)))
        return c->hipfail(e, "TCP segments");
    size_t tmp = 0;
    pv_tcp_sort(nullptr, &tmp, c->d_tkey[0], c->d_tkey[1], c->d_tval[0], c->d_tval[1], need, st);
    c->tsort_tmp_bytes = std::max<size_t>(tmp, 256);
    if (!hip_ok(e = hipMalloc(&c->d_tsort_tmp, c->tsort_tmp_bytes))) return c->hipfail(e, "TCP sort scratch");
    c->tseg_cap = (uint32_t)need;
    return 0;
}

// The TCP stage of a batch: its segments (n_seg, seg_bytes payload) through reassembly and
// framing into message records. d_offs / n: the whole batch. With want_ords the messages'
// (ord, second) pairs come back for the DNS shift plan.
int tcp_stage(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n, uint32_t n_seg, uint64_t seg_bytes,
              uint32_t now_sec, bool want_ords, hipStream_t st)
{
    c->tcp_nmsg = 0;
    c->tcp_ords.clear();
    if (n_seg > c->tseg_cap)
        return c->fail(PV_ECAPACITY, "%u DNS-over-TCP segments in one batch exceed the capacity %u (max_records)", n_seg,
                       c->tseg_cap);
    const bool eoc = c->eoc_stage && n > 0;
    c->eoc_stage = false;
    if (n_seg == 0 && !c->tcp_active) return 0;
    if (int rc = tcp_alloc(c)) return rc;
    hipError_t e;
    // bounds of this stage's output: every byte a flow can deliver (payloads, carried bytes,
    // missing-data texts) lands in at most one message record, reserved at most three times
    const uint64_t B = seg_bytes + c->carry_used + 32ull * (n_seg + c->carry_used / 8);
    if (int rc = PV_GROW(c, c->d_marena, c->marena_cap, 3 * B + 44 * (B / 17 + 2ull * n_seg) + 4096 + PV_RECS_PAD, "TCP message arena"))
        return rc;
    uint64_t fcap = c->frag_cap;
    if (int rc = PV_GROW(c, c->d_frags, fcap, n_seg + c->carry_used / 8 + 64, "TCP fragment pool")) return rc;
    c->frag_cap = (uint32_t)std::min<uint64_t>(fcap, 0xffffffffull);
    const uint32_t out = c->carry_cur ^ 1;
    if (int rc = PV_GROW(c, c->d_carry[out], c->carry_cap[out], 2 * B + 8 * (n_seg + c->carry_used / 8) + 4096, "TCP carry arena"))
        return rc;
    if (!c->d_carry[c->carry_cur]) {
        if (int rc = PV_GROW(c, c->d_carry[c->carry_cur], c->carry_cap[c->carry_cur], 4096, "TCP carry arena")) return rc;
    }
    c->tcp_stage++;
    PvTcpParams &T = *c->h_tparams;
    memset(&T, 0, sizeof T);
    T.seg = c->d_tseg;
    T.skey = c->d_tkey[1];
    T.sval = c->d_tval[1];
    T.n_seg = n_seg;
    T.stage = c->tcp_stage;
    T.now_sec = now_sec;
    T.flow_cap_log2 = c->flow_cap_log2;
    T.flows = c->d_flows;
    T.run_flow = c->d_run_flow;
    T.tmask = c->d_tmask;
    T.tpm = c->d_tpm;
    T.lt_carry = c->d_tcpcnt + PVT_WORDS;
    T.recs = d_recs;
    T.offs = d_offs;
    T.n_tiles = (uint32_t)((n + 63) / 64);
    T.ts_nano = c->cfg.ts_nano;
    T.carry_in = c->d_carry[c->carry_cur];
    T.carry_out = c->d_carry[out];
    T.carry_cap = c->carry_cap[out];
    T.clist_in = c->d_clist[c->carry_cur];
    T.n_clist_in = c->n_clist;
    T.clist_out = c->d_clist[out];
    T.frags = c->d_frags;
    T.frag_cap = c->frag_cap;
    T.marena = c->d_marena;
    T.marena_cap = c->marena_cap;
    T.moffs = c->d_moffs;
    T.mq = c->d_tmq;
    T.mq_cap = c->tmsg_cap;
    T.cnt = c->d_tcpcnt;
    flush_fills(c);
    const PvTcpParams *dT = c->d_tparams;
    uint32_t blocks = (n_seg + 255) / 256;
    // one run of the stage's kernels (dry: the exact LRU replay's recording run)
    auto run = [&](bool dry) -> int {
        T.dry = dry ? 1u : 0u;
        if (!hip_ok(e = hipMemsetAsync(c->d_tcpcnt, 0, PVT_WORDS * 4, st)) ||
            !hip_ok(e = upload_params(c->d_tparams, c->h_tparams, sizeof T, st)))
            return c->hipfail(e, "TCP stage upload");
        hipLaunchKernelGGL(pv_tcp_scan, dim3(1), dim3(1024), 0, st, dT);
        if (n_seg) {
            {
                hipLaunchKernelGGL(pv_tcp_keys, dim3(blocks), dim3(256), 0, st, (const PvTcpSeg *)c->d_tseg, n_seg, c->d_tkey[0],
                                   c->d_tval[0]);
                size_t tmp = c->tsort_tmp_bytes;
                if (!hip_ok(e = pv_tcp_sort(c->d_tsort_tmp, &tmp, c->d_tkey[0], c->d_tkey[1], c->d_tval[0], c->d_tval[1], n_seg, st)))
                    return c->hipfail(e, "TCP segment sort");
            }
            hipLaunchKernelGGL(pv_tcp_lookup, dim3(blocks), dim3(256), 0, st, dT);
            hipLaunchKernelGGL(pv_tcp_insert, dim3(blocks), dim3(256), 0, st, dT);
            hipLaunchKernelGGL(pv_tcp_flow, dim3(blocks), dim3(256), 0, st, dT);
            if (c->n_clist && !dry) hipLaunchKernelGGL(pv_tcp_migrate, dim3((c->n_clist + 255) / 256), dim3(256), 0, st, dT);
        }
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch TCP stage");
        return 0;
    };
    T.exact = c->tcp_exact_on() ? 1u : 0u;
    if (T.exact && n_seg) {
        // the exact LRU mode: record the segments' LRU events, replay the LRU list on the host,
        // then run the stage with the closes it found (close-only segments behind the batch's)
        if (int rc = PV_GROW(c, c->d_lru_ev, c->lru_ev_cap, 3ull * n_seg, "TCP LRU events")) return rc;
        T.lru_ev = c->d_lru_ev;
        T.fclose = nullptr;
        if (int rc = run(true)) return rc;
        std::vector<uint64_t> skey(n_seg);
        std::vector<uint32_t> sval(n_seg), ev(3ull * n_seg);
        if (!hip_ok(e = hipMemcpyAsync(skey.data(), c->d_tkey[1], (size_t)n_seg * 8, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(sval.data(), c->d_tval[1], (size_t)n_seg * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(ev.data(), c->d_lru_ev, ev.size() * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "TCP LRU events");
        std::vector<uint32_t> fclose(3ull * n_seg, PVT_FCLOSE_NONE), extra_fc;
        std::vector<PvTcpSeg> extra;
        tcp_lru_replay(c, skey, sval, ev, fclose, extra, extra_fc);
        if (!extra.empty()) {
            if (n_seg + extra.size() > c->tseg_cap)
                return c->fail(PV_ECAPACITY, "%u TCP segments and %zu LRU closes in one batch exceed the capacity %u (max_records)",
                               n_seg, extra.size(), c->tseg_cap);
            fclose.insert(fclose.end(), extra_fc.begin(), extra_fc.end());
            if (!hip_ok(e = hipMemcpyAsync(c->d_tseg + n_seg, extra.data(), extra.size() * sizeof(PvTcpSeg), hipMemcpyHostToDevice, st)))
                return c->hipfail(e, "TCP LRU closes");
            n_seg += (uint32_t)extra.size();
            T.n_seg = n_seg;
            blocks = (n_seg + 255) / 256;
        }
        if (int rc = PV_GROW(c, c->d_fclose, c->fclose_cap, 3ull * n_seg, "TCP LRU closes")) return rc;
        if (!hip_ok(e = hipMemcpyAsync(c->d_fclose, fclose.data(), fclose.size() * 4, hipMemcpyHostToDevice, st)))
            return c->hipfail(e, "TCP LRU closes");
        c->tcp_stage++;
        T.stage = c->tcp_stage;
        T.lru_ev = nullptr;
        T.fclose = c->d_fclose;
        if (!hip_ok(e = hipStreamSynchronize(st))) return c->hipfail(e, "TCP LRU closes");
    }
    if (eoc) {
        // TcpReassembly::closeAllConnections after the capture's last record (PcapInputStream.cpp:522,
        // :244 on stop): a close segment for every open connection, with the last record's time and
        // the direction the input cached for it (_packet_dir_cache, :399-416)
        const uint32_t ncap = 1u << c->flow_cap_log2;
        const uint64_t ncand = (uint64_t)ncap + n_seg;
        uint32_t set_log2 = 4;
        while ((1ull << set_log2) < 2 * ncand) set_log2++;
        if (ncand > c->eoc_cap) {
            if (c->d_eoc) (void)hipFree(c->d_eoc);
            c->d_eoc = nullptr;
            c->eoc_cap = 0;
            if (!hip_ok(e = hipMalloc(&c->d_eoc, (size_t)ncand * sizeof(PvTcpSeg)))) return c->hipfail(e, "TCP end-of-capture segments");
            c->eoc_cap = ncand;
        }
        if (!c->d_eoc_cnt && !hip_ok(e = hipMalloc(&c->d_eoc_cnt, 4))) return c->hipfail(e, "TCP end-of-capture segments");
        uint64_t *d_set = nullptr;
        struct SetFree {
            uint64_t *&p;
            ~SetFree() { if (p) (void)hipFree(p); }
        } set_free{d_set};
        if (!hip_ok(e = hipMalloc((void **)&d_set, (size_t)8 << set_log2)) ||
            !hip_ok(e = hipMemsetAsync(d_set, 0, (size_t)8 << set_log2, st)))
            return c->hipfail(e, "TCP end-of-capture key set");
        uint32_t lo = 0;
        uint8_t rec[16 + 512];
        memset(rec, 0, sizeof rec);
        if (!hip_ok(e = hipMemcpyAsync(&lo, d_offs + (n - 1), 4, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)) ||
            !hip_ok(e = hipMemcpyAsync(rec, d_recs + lo, 16, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "last record");
        uint32_t hdr[4];
        memcpy(hdr, rec, 16);
        const uint32_t cap = std::min<uint32_t>(hdr[2], 512);
        if (cap && (!hip_ok(e = hipMemcpyAsync(rec + 16, d_recs + lo + 16, cap, hipMemcpyDeviceToHost, st)) ||
                    !hip_ok(e = hipStreamSynchronize(st))))
            return c->hipfail(e, "last record");
        PvParams P;
        params_common(c, P, d_recs, d_offs, n);
        pvname::Parsed o;
        pvname::parse_record(pvname::HostRecs{rec, 16 + (size_t)cap}, pvname::parse_cfg(P), P, 0, o);
        const uint32_t usec = c->cfg.ts_nano ? hdr[1] / 1000u : hdr[1];
        if (!hip_ok(e = hipMemsetAsync(c->d_eoc_cnt, 0, 4, st)) || !hip_ok(e = upload_params(c->d_tparams, c->h_tparams, sizeof T, st)))
            return c->hipfail(e, "TCP end of capture");
        hipLaunchKernelGGL(pv_tcp_eoc, dim3((uint32_t)((ncand + 255) / 256)), dim3(256), 0, st, dT, (const PvTcpSeg *)c->d_tseg, n_seg,
                           d_set, (uint32_t)((1ull << set_log2) - 1), c->d_eoc, c->d_eoc_cnt, (uint32_t)(n - 1), hdr[0], usec,
                           (uint32_t)o.dir);
        uint32_t ne = 0;
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(&ne, c->d_eoc_cnt, 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "TCP end of capture");
        if (ne) {
            if (int rc = tcp_grow_segs(c, (uint64_t)n_seg + ne, n_seg, st)) return rc;
            if (!hip_ok(e = hipMemcpyAsync(c->d_tseg + n_seg, c->d_eoc, (size_t)ne * sizeof(PvTcpSeg), hipMemcpyDeviceToDevice, st)))
                return c->hipfail(e, "TCP end of capture");
            if (T.fclose) {
                // (the exact LRU mode's closes are per segment: none for these)
                std::vector<uint32_t> none(3ull * ne, PVT_FCLOSE_NONE);
                if (int rc = PV_GROW(c, c->d_fclose, c->fclose_cap, 3ull * (n_seg + ne), "TCP LRU closes")) return rc;
                if (!hip_ok(e = hipMemcpyAsync(c->d_fclose + 3ull * n_seg, none.data(), none.size() * 4, hipMemcpyHostToDevice, st)) ||
                    !hip_ok(e = hipStreamSynchronize(st)))
                    return c->hipfail(e, "TCP end of capture");
                T.fclose = c->d_fclose;
            }
            n_seg += ne;
            T.n_seg = n_seg;
            T.seg = c->d_tseg;
            T.skey = c->d_tkey[1];
            T.sval = c->d_tval[1];
            T.run_flow = c->d_run_flow;
            blocks = (n_seg + 255) / 256;
        }
    }
    if (int rc = run(false)) return rc;
    if (!hip_ok(e = hipMemcpyAsync(c->h_tcpcnt, c->d_tcpcnt, PVT_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "TCP stage");
    c->tcp_active = true;
    if (!n_seg) return 0; // the TCP record seconds advanced; no flow moved
    const uint32_t *k = c->h_tcpcnt;
    if (k[PVT_FLAGS] & PVT_F_TABLE)
        return c->fail(PV_ECAPACITY, "TCP flow table full (%u entries)", 1u << c->flow_cap_log2);
    if (k[PVT_FLAGS] & PVT_F_MSGS)
        return c->fail(PV_ECAPACITY, "more than %u DNS-over-TCP messages in one batch", c->tmsg_cap);
    if (k[PVT_FLAGS] & (PVT_F_ARENA | PVT_F_CARRY | PVT_F_FRAGS))
        return c->fail(PV_ECAPACITY, "TCP stage buffer overflow (flags 0x%x)", k[PVT_FLAGS]);
    c->tcp_nmsg = k[PVT_NMSG];
    c->n_clist = k[PVT_NCARRY];
    c->carry_used = k[PVT_CARRY];
    c->carry_cur = out;
    if (const char *dp = getenv("PV_TCP_DUMP")) {
        // debug: the batch's messages as "record sub length txid stamp_sec stamp_nsec"
        std::vector<uint32_t> items((size_t)c->tcp_nmsg * 8);
        std::vector<uint8_t> arena(k[PVT_ARENA]);
        if (c->tcp_nmsg) hipMemcpy(items.data(), c->d_tmq, items.size() * 4, hipMemcpyDeviceToHost);
        if (!arena.empty()) hipMemcpy(arena.data(), c->d_marena, arena.size(), hipMemcpyDeviceToHost);
        if (FILE *f = fopen(dp, "a")) {
            for (uint32_t q = 0; q < c->tcp_nmsg; q++) {
                const uint32_t *it = &items[(size_t)q * 8];
                const uint32_t mo = it[1];
                fprintf(f, "%llu %u %u %u %u %u\n", (unsigned long long)(c->records_seen + it[7] / 4), it[7] & 3, it[2] & 0xffff,
                        mo + 1 < arena.size() ? (arena[mo] << 8 | arena[mo + 1]) : 0u, it[5], it[6]);
            }
            fclose(f);
        }
    }
    if (want_ords && c->tcp_nmsg) {
        std::vector<uint32_t> items((size_t)c->tcp_nmsg * 8);
        if (!hip_ok(e = hipMemcpy(items.data(), c->d_tmq, items.size() * 4, hipMemcpyDeviceToHost)))
            return c->hipfail(e, "TCP message order");
        c->tcp_ords.resize(c->tcp_nmsg);
        for (uint32_t q = 0; q < c->tcp_nmsg; q++) c->tcp_ords[q] = {items[(size_t)q * 8 + 7], (int64_t)items[(size_t)q * 8 + 5]};
        std::sort(c->tcp_ords.begin(), c->tcp_ords.end());
        c->tcp_items.resize(c->tcp_nmsg);
        for (uint32_t q = 0; q < c->tcp_nmsg; q++) c->tcp_items[q] = {items[(size_t)q * 8 + 7], q};
        std::sort(c->tcp_items.begin(), c->tcp_items.end());
    }
    return 0;
}

// The TCP DNS pass of a span: the batch's messages with ord in [4 * a, 4 * b), events in
// the workgroup regions behind the span's grid; returns the workgroups it used
uint32_t tcp_pass(pv_ctx *c, const PvParams &P, uint64_t a, uint64_t b, hipStream_t st, PvParams *d_slot)
{
    if (!c->tcp_nmsg) return 0;
    PvParams Q = P;
    Q.recs = c->d_marena;
    Q.offs = c->d_moffs;
    Q.linktype = 101;
    Q.dq = c->d_tmq;
    Q.sfx_of = c->d_tsfx;
    Q.tcp_pass = 1;
    Q.ndeep_dns = c->sample_rate < 100 ? c->d_ntcp : nullptr; // per message item (pv_dns_tcp)
    Q.tcp_emit = 0;
    Q.tcp_nmsg = c->tcp_nmsg;
    Q.ord_lo = (uint32_t)(a * 4);
    Q.ord_hi = (uint32_t)std::min<uint64_t>(b * 4, 0xffffffffull);
    Q.ord_base = (uint32_t)(a * 4);
    const uint64_t region = (uint64_t)P.wt_per_block * 64;
    const uint32_t gt = (uint32_t)((c->tcp_nmsg + region - 1) / region);
    *d_slot = Q; // pinned host staging of the second parameter block
    hipMemcpyAsync(c->d_params + 1, d_slot, sizeof Q, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(pv_dns_tcp, dim3(gt), dim3(256), 0, st, (const PvParams *)(c->d_params + 1));
    return gt;
}

// One device batch with at most PV_MAX_SHIFTS shifts of each manager. nsh / dsh: the Net and
// DNS shifts inside it (record indices relative to d_offs).
// Bounded top-N (the frequent-items sketch's purge as TopN uses it, src/Metrics.h:488-503):
// a table holding more than half its capacity after a batch has each region purged at its
// median count (pv_topn_purge); the thetas become the estimate offsets read_topn adds. The
// name arena of a purged table is compacted once its fullest partition is half used. The
// live counts are the ones read back with the batch status (names added by the transaction
// pass afterwards are counted at the next batch).
int purge_table(pv_ctx *c, uint32_t t, hipStream_t st, const PvParams *dP = nullptr);
int purge_tables(pv_ctx *c, hipStream_t st)
{
    const uint64_t tcap = 1ull << c->tcap_log2;
    for (uint32_t t = 0; t < PV_TABLES; t++) {
        if (c->h_tab_live[t] <= tcap / 2) continue;
        if (int rc = purge_table(c, t, st)) return rc;
    }
    return 0;
}

// Updates full regions could not take in this batch (PvOvf list): purge each table they belong
// to, as the sketch purges when its map is full, and insert them again, until none is left.
// Each round at least halves the live entries of every region it purges, so the rounds end.
// known: c->h_ovf already holds the words (read back with the batch status).
int drain_overflow(pv_ctx *c, hipStream_t st, bool known = false, bool *drained = nullptr, const PvParams *dP = nullptr)
{
    if (!dP) dP = c->d_params;
    hipError_t e;
    for (int round = 0;; round++) {
        uint32_t oc[2];
        if (!(known && round == 0) &&
            (!hip_ok(e = hipMemcpyAsync(c->h_ovf, c->d_ovf_cnt, 8, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st))))
            return c->hipfail(e, "top-N overflow");
        memcpy(oc, c->h_ovf, 8);
        if (!oc[0]) return 0;
        if (drained) *drained = true;
        if (oc[0] > c->ovf_cap) return c->fail(PV_ECAPACITY, "top-N overflow list full (%u updates)", oc[0]);
        if (round >= 64) return c->fail(PV_ECAPACITY, "top-N overflow not drained after %d purge rounds", round);
        for (uint32_t t = 0; t < PV_TABLES; t++)
            if ((oc[1] >> t) & 1)
                if (int rc = purge_table(c, t, st, dP)) return rc;
        if (!hip_ok(e = hipMemcpyAsync(c->d_ovf2, c->d_ovf, (size_t)oc[0] * sizeof(PvOvf), hipMemcpyDeviceToDevice, st)) ||
            !hip_ok(e = hipMemsetAsync(c->d_ovf_cnt, 0, 8, st)))
            return c->hipfail(e, "top-N overflow");
        hipLaunchKernelGGL(pv_topn_retry, dim3((oc[0] + 255) / 256), dim3(256), 0, st, dP, c->d_ovf2, oc[0]);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_topn_retry");
        c->ovf_rounds++;
    }
}

int purge_table(pv_ctx *c, uint32_t t, hipStream_t st, const PvParams *dP)
{
    if (!dP) dP = c->d_params;
    const uint32_t nreg = 1u << c->reg_log2;
    hipError_t e;
    {
        c->h_tab_live[t] = 0; // stale until the next batch reads the device count back
        hipLaunchKernelGGL(pv_topn_purge, dim3(nreg), dim3(1024), 0, st, dP, t, c->d_theta);
        std::vector<uint32_t> th(nreg);
        uint64_t tops[PV_ARENA_PARTS];
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(th.data(), c->d_theta, nreg * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(tops, c->d_arena_top + (uint64_t)t * PV_ARENA_PARTS, sizeof tops, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "top-N purge");
        std::vector<uint64_t> &ro = c->roff[t];
        ro.resize(nreg, 0);
        for (uint32_t r = 0; r < nreg; r++) ro[r] += th[r];
        c->purges++;
        const uint64_t pcap = c->arena_cap / PV_ARENA_PARTS;
        uint64_t most = 0;
        for (uint64_t u : tops) most = std::max(most, u);
        if (most <= pcap / 2) return 0;
        if (!c->d_ctmp) {
            if (!hip_ok(e = hipMalloc(&c->d_ctmp, c->arena_cap)) || !hip_ok(e = hipMalloc(&c->d_ctop, PV_ARENA_PARTS * 8)))
                return c->hipfail(e, "arena compaction scratch");
        }
        uint8_t *arena = c->d_arena + (uint64_t)t * c->arena_cap;
        if (!hip_ok(e = hipMemsetAsync(c->d_ctop, 0, PV_ARENA_PARTS * 8, st))) return c->hipfail(e, "arena compaction");
        hipLaunchKernelGGL(pv_topn_compact, dim3((uint32_t)c->cus * 8), dim3(256), 0, st, dP, t, c->d_ctmp, c->d_ctop);
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(arena, c->d_ctmp, c->arena_cap, hipMemcpyDeviceToDevice, st)) ||
            !hip_ok(e = hipMemcpyAsync(c->d_arena_top + (uint64_t)t * PV_ARENA_PARTS, c->d_ctop, PV_ARENA_PARTS * 8,
                                       hipMemcpyDeviceToDevice, st)))
            return c->hipfail(e, "arena compaction");
    }
    return 0;
}

// Records of `n` batch indices (d_idx[i * stride], PV_TCP_IDX: the TCP message arena) appended
// to the context's slow store; offs_out[i] = each record's offset there
int gather_records(pv_ctx *c, const PvParams &P, const uint32_t *d_idx, uint32_t stride, uint32_t n,
                   std::vector<uint32_t> &offs_out, hipStream_t st)
{
    offs_out.assign(n, 0);
    if (!n) return 0;
    hipError_t e;
    uint32_t *d_sz = nullptr, *d_off = nullptr;
    uint8_t *d_out = nullptr;
    struct Free { void *p[3]; ~Free() { for (void *q : p) if (q) hipFree(q); } } fr{{nullptr, nullptr, nullptr}};
    if (!hip_ok(e = hipMalloc(&d_sz, (size_t)n * 4)) || !hip_ok(e = hipMalloc(&d_off, (size_t)n * 4)))
        return c->hipfail(e, "slow store scratch");
    fr.p[0] = d_sz; fr.p[1] = d_off;
    hipLaunchKernelGGL(pv_rec_sizes, dim3((n + 255) / 256), dim3(256), 0, st, P.recs, P.offs, c->d_marena, c->d_moffs, d_idx, stride,
                       n, d_sz);
    std::vector<uint32_t> sz(n);
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(sz.data(), d_sz, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "slow store sizes");
    uint64_t tot = 0;
    std::vector<uint32_t> rel(n);
    for (uint32_t i = 0; i < n; i++) { rel[i] = (uint32_t)tot; tot += sz[i]; }
    if (c->sstore.size() + tot > 0xfffffff0ull) return c->fail(PV_ECAPACITY, "deferred slow-transaction records exceed 4 GiB");
    if (!hip_ok(e = hipMalloc(&d_out, tot ? tot : 4))) return c->hipfail(e, "slow store scratch");
    fr.p[2] = d_out;
    if (!hip_ok(e = hipMemcpyAsync(d_off, rel.data(), (size_t)n * 4, hipMemcpyHostToDevice, st))) return c->hipfail(e, "slow store");
    hipLaunchKernelGGL(pv_rec_gather, dim3((n + 3) / 4), dim3(256), 0, st, P.recs, P.offs, c->d_marena, c->d_moffs, d_idx, stride, n,
                       d_off, d_out);
    const size_t base = c->sstore.size();
    c->sstore.resize(base + tot);
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(c->sstore.data() + base, d_out, tot, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "slow store");
    for (uint32_t i = 0; i < n; i++) offs_out[i] = (uint32_t)(base + rel[i]);
    return 0;
}

// Sharded top_slow (pv_set_slow_defer): the batch's slow-transaction candidates (every valid,
// deep transaction of known direction: the resolve was given no threshold) and its new orphan
// stubs are kept with their response records; pv_slow_finish checks them against the
// thresholds of the whole stream (DnsMetricsManager::on_period_shift, dns/v1/DnsStreamHandler.h:
// 252-267) once the ranks' values are merged.
int defer_slow(pv_ctx *c, const PvParams &P, hipStream_t st)
{
    hipError_t e;
    uint32_t nv[4];
    if (!hip_ok(e = hipMemcpyAsync(nv, c->d_nvals, 16, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "deferred candidates");
    // period k of the span: the k-th DNS shift after the live one (the window bookkeeping of
    // this span's shifts runs after the transaction stage, so the slots' ordinals are not
    // recorded yet)
    (void)P;
    auto ord_of = [&](uint32_t period) -> uint64_t { return c->dns.ordinal + period; };
    if (nv[1]) {
        std::vector<PvXValid> v(nv[1]);
        std::vector<uint32_t> offs;
        if (!hip_ok(e = hipMemcpy(v.data(), c->d_valid, v.size() * sizeof(PvXValid), hipMemcpyDeviceToHost)))
            return c->hipfail(e, "deferred candidates");
        if (int rc = gather_records(c, P, reinterpret_cast<const uint32_t *>(c->d_valid), sizeof(PvXValid) / 4, nv[1], offs, st))
            return rc;
        for (uint32_t i = 0; i < nv[1]; i++)
            if (v[i].dir < 2 || v[i].dir >= 4) // v1 directions, DNS v2's 4 + transaction direction
                c->scands.push_back(pv_ctx::SlowCand{ord_of(v[i].period), v[i].us, offs[i], v[i].dir, (uint8_t)((v[i].idx & PV_TCP_IDX) != 0)});
        const uint32_t zero = 0;
        if (!hip_ok(e = hipMemcpyAsync(c->d_nvals + 1, &zero, 4, hipMemcpyHostToDevice, st))) return c->hipfail(e, "deferred candidates");
    }
    const uint32_t no = std::min(nv[3], c->orph_cap);
    if (nv[3] > c->orph_cap) return c->fail(PV_ECAPACITY, "%u shard-edge stubs exceed the stub capacity", nv[3]);
    if (no > c->orph_done) {
        const uint32_t k = no - c->orph_done;
        std::vector<PvXEvent> o(k);
        std::vector<int64_t> oo(k, 0);
        if (!hip_ok(e = hipMemcpy(o.data(), c->d_orph + c->orph_done, (size_t)k * sizeof(PvXEvent), hipMemcpyDeviceToHost)) ||
            (c->d_orph_ord && !hip_ok(e = hipMemcpy(oo.data(), c->d_orph_ord + c->orph_done, (size_t)k * 8, hipMemcpyDeviceToHost))))
            return c->hipfail(e, "orphan stubs");
        // the records of the responses (an edge pair's top_slow candidate needs its name)
        std::vector<uint32_t> ridx;
        for (auto &x : o)
            if (x.qr) ridx.push_back(x.idx);
        std::vector<uint32_t> offs;
        if (!ridx.empty()) {
            uint32_t *d_idx = nullptr;
            if (!hip_ok(e = hipMalloc(&d_idx, ridx.size() * 4)) ||
                !hip_ok(e = hipMemcpy(d_idx, ridx.data(), ridx.size() * 4, hipMemcpyHostToDevice)))
                return c->hipfail(e, "orphan stubs");
            const int rc = gather_records(c, P, d_idx, 1, (uint32_t)ridx.size(), offs, st);
            hipFree(d_idx);
            if (rc) return rc;
        }
        size_t r = 0;
        for (uint32_t i = 0; i < k; i++) {
            const uint64_t ord = ord_of(o[i].period & 0x3f); // DNS v2 stubs: the kept flag in bit 7
            int64_t cand = -1;
            if (o[i].qr) {
                cand = (int64_t)c->sorph.size();
                c->sorph.push_back(pv_ctx::SlowCand{ord, 0, offs[r++], o[i].dir, (uint8_t)((o[i].idx & PV_TCP_IDX) != 0)});
            }
            c->stubs.push_back(pv_ctx::EdgeStub{o[i], ord, cand, oo[i]});
        }
        c->orph_done = no;
    }
    return hip_ok(e = hipStreamSynchronize(st)) ? 0 : c->hipfail(e, "deferred candidates");
}

// The DNS transaction stage of a batch (TransactionManager state across batches): a batch with
// responses or a DNS period shift pairs (sort + resolve) its nev_b events together with the
// queries carried in; a batch of queries only just appends them to the carried list. Also the
// heartbeat's DNS shift (nev_b = 0, one shift): the carried queries the shift purges time out
// in the new live bucket, the rest carry on.
// The rank values quantile_at(values, r) gives for each kind of PvXvSel among the transaction
// values of slot sg: the device buffer's by radix selection there (pv_xv_hist, eight passes), and
// those a drain already moved to the host (xvals_host ahead of the current device buffer's copy)
// counted into the same histograms. have[k] = the kind has values. Synchronises.
int xv_select(pv_ctx *c, uint32_t sg, double r, bool have[PV_XV_SEL], uint64_t out[PV_XV_SEL])
{
    hipError_t e;
    if (!c->d_xvh && (!hip_ok(e = hipMalloc(&c->d_xvh, PV_XV_SEL * 256 * 4)) ||
                      !hip_ok(e = hipHostMalloc((void **)&c->h_xvh, PV_XV_SEL * 256 * 4, hipHostMallocDefault))))
        return c->hipfail(e, "threshold selection");
    auto kind_of = [](uint32_t kind) {
        return kind == XV_FROM_US ? 0 : kind == XV_TO_US ? 1 : (kind >= XV2_TIME && kind < XV2_TIME + 3) ? 2 + (int)(kind - XV2_TIME) : -1;
    };
    {
        // a value buffer that overflowed holds a truncated value set: fail as sync_xvals does
        uint32_t flags = 0, nv = 0;
        if (!hip_ok(e = hipStreamSynchronize(c->stream)) ||
            !hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost)) ||
            !hip_ok(e = hipMemcpy(&nv, c->d_nvals, 4, hipMemcpyDeviceToHost)))
            return c->hipfail(e, "threshold selection");
        if ((flags & PVF_VALUES_FULL) || nv > c->xv_cap) return c->fail(PV_ECAPACITY, "transaction value buffer full");
    }
    std::vector<uint64_t> hv[PV_XV_SEL];
    const size_t host_only = c->xvals_host.size() - c->xvals_synced;
    for (size_t i = 0; i < host_only; i++) {
        const PvXValue &v = c->xvals_host[i];
        const int k = v.slot == sg ? kind_of(v.kind) : -1;
        if (k >= 0) hv[k].push_back(v.bits);
    }
    PvXvSel sel;
    memset(&sel, 0, sizeof sel);
    uint64_t rank[PV_XV_SEL] = {0};
    for (int pass = 0; pass < 8; pass++) {
        const uint32_t shift = 56 - 8 * pass;
        if (!hip_ok(e = hipMemsetAsync(c->d_xvh, 0, PV_XV_SEL * 256 * 4, c->stream))) return c->hipfail(e, "threshold selection");
        hipLaunchKernelGGL(pv_xv_hist, dim3(std::max<uint32_t>(1u, (uint32_t)c->cus * 2)), dim3(256), 0, c->stream, c->d_xvals, c->d_nvals,
                           (uint32_t)c->xv_cap, sg, shift, sel, c->d_xvh);
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(c->h_xvh, c->d_xvh, PV_XV_SEL * 256 * 4, hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "threshold selection");
        const uint64_t hm = shift >= 56 ? 0ull : ~0ull << (shift + 8);
        for (int k = 0; k < PV_XV_SEL; k++) {
            uint64_t h[256];
            for (int b = 0; b < 256; b++) h[b] = c->h_xvh[k * 256 + b];
            for (uint64_t x : hv[k])
                if ((x & hm) == (sel.prefix[k] & hm)) h[(x >> shift) & 255]++;
            if (pass == 0) {
                uint64_t total = 0;
                for (int b = 0; b < 256; b++) total += h[b];
                have[k] = total > 0;
                const uint64_t w = (uint64_t)std::ceil(r * (double)total);
                rank[k] = w == 0 ? 0 : std::min(w - 1, total ? total - 1 : 0);
            }
            if (!have[k]) continue;
            uint64_t cum = 0;
            int b = 0;
            while (b < 255 && cum + h[b] <= rank[k]) cum += h[b++];
            rank[k] -= cum;
            sel.prefix[k] |= (uint64_t)b << shift;
        }
    }
    for (int k = 0; k < PV_XV_SEL; k++) out[k] = sel.prefix[k];
    return 0;
}

int pair_stage(pv_ctx *c, const PvParams &P, uint32_t nev_b, uint32_t nkeys, uint32_t nresp, uint64_t n, hipStream_t st,
               uint64_t ev_hi)
{
    hipError_t e;
    const bool dns_here = nev_b > 0;
    bool pair = (dns_here && (nresp > 0 || P.n_dshift > 0)) || (!dns_here && P.n_dshift > 0 && c->n_pend > 0);
    if (dns_here && !pair && (c->n_pend + nev_b > c->pend_cap || (c->n_pend && c->pend_hi + nev_b > c->ev_store_cap)))
        pair = true; // compact the carried list
    if (dns_here && !pair) {
        const uint32_t cur = c->pend_cur;
        if (c->n_pend == 0 && nkeys == nev_b) {
            // nothing carried: the batch's event store, sorted-key inputs and ECS words become the
            // carried list as they lie (pointer exchange; the next batch writes the other buffers)
            std::swap(c->d_events, c->d_pend[cur]);
            std::swap(c->d_skeys, c->d_pkeys[cur]);
            std::swap(c->d_svals, c->d_pvals[cur]);
            if (c->d_eecs) std::swap(c->d_eecs, c->d_pecs[cur]);
            c->pend_hi = ev_hi;
        } else {
            // (the key list's sentinel slots, messages without an event, are left out)
            if (!hip_ok(e = hipMemsetAsync(c->d_nvals + 2, 0, 4, st))) return c->hipfail(e, "defer counter");
            hipLaunchKernelGGL(pv_xact_defer, dim3((nkeys + 255) / 256), dim3(256), 0, st, c->d_skeys, c->d_svals,
                               c->d_events, nkeys, c->d_pend[cur], c->d_pkeys[cur], c->d_pvals[cur], (uint32_t)c->n_pend,
                               (uint32_t)c->pend_hi, c->d_eecs, c->d_pecs[cur], c->d_nvals + 2);
            if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_defer");
            c->pend_hi += nev_b;
        }
        c->n_pend += nev_b;
    }
    if (pair) {
        const uint32_t np_in = (uint32_t)c->n_pend;
        if (np_in) {
            hipLaunchKernelGGL(pv_xact_pend_in, dim3((np_in + 255) / 256), dim3(256), 0, st, c->d_skeys, c->d_svals,
                               c->d_pkeys[c->pend_cur], c->d_pvals[c->pend_cur], np_in, nkeys);
            if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_pend_in");
        }
        HP(10);
        // sorted: this batch's events and the carried queries first, the sentinel slots behind
        const uint32_t nev = nev_b + np_in;
        uint32_t threads = 256, blocks = (nev + threads - 1) / threads;
        size_t tmp = c->sort_tmp_bytes;
        if (!hip_ok(e = pv_radix_sort_pairs(c->d_sort_tmp, &tmp, c->d_skeys, c->d_skeys2, c->d_svals, c->d_svals2,
                                             (size_t)nkeys + np_in, st)))
            return c->hipfail(e, "radix sort");
        HP(11);
        PvXactParams X;
        memset(&X, 0, sizeof X);
        X.P = P;
        X.events = c->d_events;
        X.skeys = c->d_skeys2;
        X.svals = c->d_svals2;
        X.n = nev;
        X.ttl_s = c->ttl_s;
        X.ttl_ms = c->ttl_ms;
        X.quantiles = ((c->dns_groups & PV_DNS_QUANTILES) ? 1u : 0u) | ((c->dns_groups & PV_DNS_HISTOGRAMS) ? 2u : 0u);
        for (uint32_t k = 0; k <= P.n_dshift; k++) {
            X.slot_gen[k] = P.dslot_of[k] | (c->gen[P.dslot_of[k]] << 8);
            X.thr_from[k] = k == 0 && !c->slow_defer ? c->from90 : -1.0f;
            X.thr_to[k] = k == 0 && !c->slow_defer ? c->to90 : -1.0f;
            for (uint32_t d = 0; d < 3; d++) X.thr2[k][d] = k == 0 && !c->slow_defer ? c->p90_2[d] : -1.0f;
        }
        X.vals = c->d_xvals;
        X.n_vals = c->d_nvals;
        X.vals_cap = (uint32_t)c->xv_cap;
        X.valid = c->d_valid;
        X.n_valid = c->d_nvals + 1;
        X.pend = c->d_pend[c->pend_cur];
        X.pend_out = c->d_pend[c->pend_cur ^ 1];
        X.pecs = c->d_pecs[c->pend_cur];
        X.pecs_out = c->d_pecs[c->pend_cur ^ 1];
        X.pkeys_out = c->d_pkeys[c->pend_cur ^ 1];
        X.pvals_out = c->d_pvals[c->pend_cur ^ 1];
        X.n_pend_out = c->d_nvals + 2;
        X.orph = c->d_orph;
        X.n_orph = c->d_nvals + 3;
        X.orph_cap = c->orph_cap;
        X.trecs = c->d_marena;
        X.toffs = c->d_moffs;
        X.tsfx = c->d_tsfx;
        X.edge_h = c->slow_defer ? c->edge_h : 0;
        X.orph_ord = c->slow_defer && c->dns2_groups ? c->d_orph_ord : nullptr; // DNS v2 stubs
        HP(15);
        if (!hip_ok(e = hipMemsetAsync(c->d_nvals + 2, 0, 4, st))) return c->hipfail(e, "parameter upload");
        HP(16);
        if (!hip_ok(e = (*c->h_xparams = X, upload_params(c->d_xparams, c->h_xparams, sizeof X, st))))
            return c->hipfail(e, "parameter upload");
        HP(17);
        hipLaunchKernelGGL(pv_xact_resolve, dim3(blocks), dim3(threads), 0, st, (const PvXactParams *)c->d_xparams);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_resolve");
        HP(18);
        // (the resolve kernel also moves the queries still open to the carried list: pv_xact_carry's work)
        if (c->slow_defer) {
            if (int rc = defer_slow(c, P, st)) return rc;
        } else if (P.n_dshift > 0 && ((c->dns_groups & PV_DNS_QUANTILES) || (c->dns2_groups & PV_DNS2_XACT_TIMES))) {
            // on_period_shift: slow thresholds = p90 of the bucket that just closed
            // (dns/v1/DnsStreamHandler.h:259-266); kept when that bucket had none
            HP(19);
            for (uint32_t k = 1; k <= P.n_dshift; k++) {
                const uint32_t sg = P.dslot_of[k - 1] | (c->gen[P.dslot_of[k - 1]] << 8);
                bool have[PV_XV_SEL];
                uint64_t q[PV_XV_SEL];
                if (int rc = xv_select(c, sg, 0.90, have, q)) return rc;
                if (have[0]) c->from90 = (float)q[0];
                if (have[1]) c->to90 = (float)q[1];
                X.thr_from[k] = c->from90;
                X.thr_to[k] = c->to90;
                // DNS v2: per direction (dns/v2/DnsStreamHandler.h:440-453)
                for (uint32_t d = 0; d < 3; d++) {
                    if (have[2 + d]) c->p90_2[d] = (float)q[2 + d];
                    X.thr2[k][d] = c->p90_2[d];
                }
            }
            uint32_t nvalid = 0;
            if (!hip_ok(e = hipMemcpy(&nvalid, c->d_nvals + 1, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "valid count");
            if (nvalid) {
                if (!hip_ok(e = (*c->h_xparams = X, upload_params(c->d_xparams, c->h_xparams, sizeof X, st))))
                    return c->hipfail(e, "parameter upload");
                hipLaunchKernelGGL(pv_xact_slow, dim3((nvalid + 255) / 256), dim3(256), 0, st,
                                   (const PvXactParams *)c->d_xparams, nvalid);
                if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_slow");
            }
            uint32_t zero = 0;
            hipMemcpyAsync(c->d_nvals + 1, &zero, 4, hipMemcpyHostToDevice, st);
            hipStreamSynchronize(st);
        }
        HP(12);
        uint32_t nv3[3] = {0, 0, 0};
        if (!hip_ok(e = hipMemcpyAsync(nv3, c->d_nvals, 12, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "carried queries");
        const uint32_t npo = nv3[2];
        uint32_t vflags = 0;
        if (!hip_ok(e = hipMemcpy(&vflags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
        if ((vflags & PVF_VALUES_FULL) || nv3[0] > c->xv_cap) return c->fail(PV_ECAPACITY, "transaction value buffer full");
        // a batch pushes at most two values per response (time + ratio), so keep 2 x max_records free
        if (c->xv_cap - nv3[0] < 2ull * c->max_records) {
            // less than that room: the device value buffer doubles while it stays
            // within PV_XV_BUDGET_MB (HBM is plentiful; a copy inside HBM instead of a read-back
            // of every value inside the stream), else it drains to the host copy and every batch
            // then has the whole capacity (at most two values per response)
            const uint64_t grow = c->xv_cap * 2;
            const char *bv = getenv("PV_XV_BUDGET_MB");
            const uint64_t budget = (bv ? strtoull(bv, nullptr, 10) : 4096ull) << 20;
            PvXValue *nb = nullptr;
            if (grow <= 0xffffffffull && grow * sizeof(PvXValue) <= budget && hip_ok(hipMalloc(&nb, grow * sizeof(PvXValue)))) {
                if (!hip_ok(e = hipMemcpyAsync(nb, c->d_xvals, (size_t)nv3[0] * sizeof(PvXValue), hipMemcpyDeviceToDevice, st)) ||
                    !hip_ok(e = hipStreamSynchronize(st)))
                    return c->hipfail(e, "value buffer growth");
                hipFree(c->d_xvals);
                c->d_xvals = nb;
                c->xv_cap = grow;
            } else {
                if (int rc = sync_xvals(c)) return rc;
                c->xvals_synced = 0;
                if (!hip_ok(e = hipMemsetAsync(c->d_nvals, 0, 4, st))) return c->hipfail(e, "value buffer drain");
            }
        }
        if (npo > c->pend_cap) return c->fail(PV_ECAPACITY, "%u open DNS queries exceed the carried-list capacity", npo);
        c->n_pend = npo;
        c->pend_hi = npo;
        c->pend_cur ^= 1;
        c->pend_base = (int64_t)(c->records_seen + n) - 1;
        HP(13);
    }

    return 0;
}

// the per-message bitmaps of deep sampling (filtered, not deep), for nmsg messages
int tcp_bits_alloc(pv_ctx *c, uint32_t nmsg)
{
    if (nmsg + 64 <= c->tmsg_bits_cap) return 0;
    for (void *p : {(void *)c->d_tfbits, (void *)c->d_ntcp}) if (p) hipFree(p);
    for (void *p : {(void *)c->h_tfbits, (void *)c->h_ntcp}) if (p) hipHostFree(p);
    c->d_tfbits = c->h_tfbits = nullptr;
    c->d_ntcp = c->h_ntcp = nullptr;
    c->tmsg_bits_cap = 0;
    const uint64_t cap = (uint64_t)nmsg + 4096;
    hipError_t e;
    if (!hip_ok(e = hipMalloc(&c->d_tfbits, (cap / 64 + 2) * 8)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_tfbits, (cap / 64 + 2) * 8, hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_ntcp, (cap / 32 + 64) * 4)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_ntcp, (cap / 32 + 64) * 4, hipHostMallocDefault)))
        return c->hipfail(e, "deep sampling message bitmaps");
    c->tmsg_bits_cap = cap;
    return 0;
}

// which of the batch's DNS-over-TCP messages _filtering rejects (pv_dns_tcp_filter) into
// c->h_tfbits (synchronises)
int tcp_filter_bits(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n, hipStream_t st)
{
    const uint32_t nmsg = c->tcp_nmsg;
    if (!nmsg) return 0;
    if (int rc = tcp_bits_alloc(c, nmsg)) return rc;
    PvParams Q;
    params_common(c, Q, d_recs, d_offs, n);
    Q.recs = c->d_marena;
    Q.offs = c->d_moffs;
    Q.linktype = 101;
    Q.dq = c->d_tmq;
    Q.tcp_nmsg = nmsg;
    Q.fbits = c->d_tfbits;
    c->h_params[1] = Q;
    hipError_t e;
    if (!hip_ok(e = upload_params(c->d_params + 1, c->h_params + 1, sizeof Q, st)))
        return c->hipfail(e, "parameter upload");
    const uint32_t tiles = (nmsg + 63) / 64;
    hipLaunchKernelGGL(pv_dns_tcp_filter, dim3(std::min<uint32_t>((tiles + 3) / 4, (uint32_t)c->cus * 8)), dim3(256), 0, st,
                       (const PvParams *)(c->d_params + 1));
    if (!hip_ok(e = hipGetLastError()) ||
        !hip_ok(e = hipMemcpyAsync(c->h_tfbits, c->d_tfbits, (size_t)tiles * 8, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "DNS-over-TCP filter prescan");
    return 0;
}

int process_span(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_boffs, uint64_t a, uint64_t n, uint64_t rec_bytes,
                 const std::vector<Shift> &nsh, const std::vector<Shift> &dsh, uint32_t first_sec, hipStream_t st)
{
    const uint32_t np = c->cfg.num_periods;
    const uint32_t *d_offs = d_boffs + a;
    PvParams P;
    params_common(c, P, d_recs, d_offs, n);
    // a batch with no TCP stage ahead of it is one span: its Net pass emits the TCP segments
    // and the tile masks of its TCP records (zeroed here; the pass stores non-zero masks only)
    P.tcp_emit = c->tcp_pre ? 0u : (c->tcp_exact_on() ? 7u : 1u);
    if (P.tcp_emit) launch_fill64(c, c->d_tmask, (n + 63) / 64, 0);
    P.gbase = c->global_base + c->records_seen;
    if (c->slow_defer && !c->edge_h) c->edge_h = (int64_t)first_sec + c->ttl_s + 61;
    if (c->sample_rate < 100) {
        // AbstractMetricsManager::new_event (:318-333): one draw per event of each manager, in
        // stream order. Net events are the records. DNS events are the DNS-port UDP records the
        // input predicates pass and the DNS-over-TCP messages (their order: record * 4 + the
        // message's rank); an event _filtering rejects is process_filtered, new_event(stamp,
        // false): no draw, the manager's last flag (dns/v1/DnsStreamHandler.cpp:1341-1375)
        const uint64_t words = n / 32 + 64; // padded: inactive lanes of the last tile read in bounds
        hipError_t e;
        if (words > c->ndeep_words) {
            if (c->d_ndeep) hipFree(c->d_ndeep);
            if (c->h_ndeep) hipHostFree(c->h_ndeep);
            c->d_ndeep = nullptr;
            c->h_ndeep = nullptr;
            c->ndeep_words = 0;
            if (!hip_ok(e = hipMalloc(&c->d_ndeep, words * 8)) || !hip_ok(e = hipHostMalloc((void **)&c->h_ndeep, words * 8, hipHostMallocDefault)))
                return c->hipfail(e, "deep sampling bitmaps");
            c->ndeep_words = words;
        }
        const bool filt = c->f_flags != 0;
        if (filt && !c->d_fbits) {
            const size_t fw = (size_t)(c->max_records / 64 + 2);
            if (!hip_ok(e = hipMalloc(&c->d_fbits, fw * 8)) || !hip_ok(e = hipHostMalloc((void **)&c->h_fbits, fw * 8, hipHostMallocDefault)))
                return c->hipfail(e, "deep sampling filter bits");
        }
        uint32_t tseg[2];
        if (int rc = dns_prescan(c, d_recs, d_offs, n, st, false, tseg, filt)) return rc;
        // the span's messages (ord in [4a, 4(a + n))), and which of them are filtered
        const uint32_t nmsg = c->tcp_nmsg;
        if (nmsg) {
            if (int rc = tcp_bits_alloc(c, nmsg)) return rc;
            if (filt)
                if (int rc = tcp_filter_bits(c, d_recs, d_offs, n, st)) return rc;
            memset(c->h_ntcp, 0, ((size_t)nmsg / 32 + 1) * 4);
        }
        uint32_t *hn = c->h_ndeep, *hd = c->h_ndeep + words;
        memset(hn, 0, words * 8);
        auto dns_draw = [&](bool filtered) {
            if (!filtered) c->dns_deep_now = c->draws_dns.next(c->sample_rate);
            return c->dns_deep_now;
        };
        const uint64_t olo = a * 4, ohi = (a + n) * 4;
        auto it = std::lower_bound(c->tcp_items.begin(), c->tcp_items.end(), std::make_pair(olo, 0u));
        c->draws_net.take_not_deep(c->sample_rate, hn, n);
        // the DNS events in stream order: each DNS-port UDP record, then the messages a TCP
        // record completes (ord (a + i) * 4 + sub) after the records before it
        auto tcp_upto = [&](uint64_t rec_end) {
            for (; it != c->tcp_items.end() && it->first < ohi && (it->first >> 2) < a + rec_end; ++it) {
                const uint32_t q = it->second;
                const bool f = filt && ((c->h_tfbits[q >> 6] >> (q & 63)) & 1);
                if (!dns_draw(f)) c->h_ntcp[q >> 5] |= 1u << (q & 31);
            }
        };
        for (uint64_t w = 0; w < (n + 63) / 64; w++) {
            uint64_t m = c->h_dbits[w];
            if (w == (n - 1) / 64 && n % 64) m &= (1ull << (n % 64)) - 1;
            while (m) {
                const uint64_t i = w * 64 + __builtin_ctzll(m);
                m &= m - 1;
                tcp_upto(i);
                const bool f = filt && ((c->h_fbits[i >> 6] >> (i & 63)) & 1);
                if (!dns_draw(f)) hd[i >> 5] |= 1u << (i & 31);
            }
        }
        tcp_upto(n);
        if (!hip_ok(e = hipMemcpyAsync(c->d_ndeep, c->h_ndeep, words * 8, hipMemcpyHostToDevice, st)) ||
            (nmsg && !hip_ok(e = hipMemcpyAsync(c->d_ntcp, c->h_ntcp, ((size_t)nmsg / 32 + 1) * 4, hipMemcpyHostToDevice, st))))
            return c->hipfail(e, "deep sampling bitmaps");
        P.ndeep_net = c->d_ndeep;
        P.ndeep_dns = c->d_ndeep + words;
    }
    // Net periods and slots: period 0 -> the live bucket, each shift -> the next ordinal's slot
    P.n_shift = (uint32_t)nsh.size();
    for (size_t k = 0; k < nsh.size(); k++) { P.thresh[k] = nsh[k].sec; P.pstart[k] = nsh[k].idx; }
    P.skip_before = P.n_shift + 1 > np ? P.n_shift + 1 - np : 0;
    for (uint32_t k = 0; k <= P.n_shift; k++) {
        P.slot_of[k] = c->net.slot_at(k);
        if (k) clear_part(c, PART_NET, P.slot_of[k]);
    }
    // DNS periods and slots, from the DNS manager's own shifts
    P.n_dshift = (uint32_t)dsh.size();
    for (size_t k = 0; k < dsh.size(); k++) { P.dthresh[k] = dsh[k].sec; P.dpos[k] = (uint32_t)dsh[k].ord; }
    P.dskip_before = P.n_dshift + 1 > np ? P.n_dshift + 1 - np : 0;
    for (uint32_t k = 0; k <= P.n_dshift; k++) {
        P.dslot_of[k] = c->dns.slot_at(k);
        if (k) clear_part(c, PART_DNS, P.dslot_of[k]);
    }
    P.sum = c->d_sum;
    P.cpc = c->d_cpc;
    P.tkeys = c->d_tkeys;
    P.tcnt = c->d_tcnt;
    P.taux = c->d_taux;
    P.tcap_log2 = c->tcap_log2;
    P.arena = c->d_arena;
    P.arena_top = c->d_arena_top;
    P.arena_cap = c->arena_cap;
    P.tab_live = c->d_tab_live; // global_add counts the entries it creates
    P.events = c->d_events;
    P.eecs = c->d_eecs;
    P.ekeys = c->d_ekeys;
    P.blk_events = c->d_blk_events;
    P.skeys = c->d_skeys;
    P.svals = c->d_svals;
    P.n_events = c->d_status + ST_NEV; // [0] events, [1] responses (ST_NRESP)
    P.n_keys = c->d_status + ST_NKEYS;
    P.n_dns = c->d_status + ST_NDNS;
    P.n_slow = c->d_status + ST_NSLOW;
    P.want_events = ((c->dns_groups & PV_DNS_TRANSACTIONS) || c->dns2_groups) ? 1 : 0;
    // sort ranks: carried queries 0, this batch's records from records_seen - pend_base on
    if (c->n_pend == 0) c->pend_base = (int64_t)c->records_seen - 1;
    if ((uint64_t)((int64_t)(c->records_seen + n) - c->pend_base) >= 0x3fffffffull)
        return c->fail(PV_ECAPACITY, "open DNS queries carried over more than 2^30 records without a response");
    P.ekey_base = (uint32_t)((int64_t)c->records_seen - c->pend_base);
    P.flags = c->d_status + ST_FLAGS;
    launch_fill32(c, c->d_status, ST_ALLOC, 0);
    hipError_t e;
    const uint64_t tiles = (n + 63) / 64; // 64-record wave tiles
    // persistent grid: exactly the workgroups that are resident at once (LDS/VGPR
    // occupancy), each owning a contiguous run of wave tiles
    // (a batch after one that was mostly DNS messages takes four ranges per CU: the DNS pass,
    // combine and merge of such batches gain from the finer partition, C3 2.16 -> 2.11 ms, while
    // Net-heavy batches lose, C2 0.450 -> 0.465; profiles/r5/experiments/r5oo)
    const int wgcu = !c->wg_forced && c->dns_heavy ? std::max(c->wg_per_cu, 4) : c->wg_per_cu;
    uint32_t grid = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(tiles, (uint64_t)c->cus * wgcu), PV_MAX_GRID);
    P.wt_per_block = (uint32_t)((tiles + grid - 1) / grid);
    P.rec_bytes = rec_bytes;
    {
        static const char *dbg = getenv("PV_DEBUG_STAGES");
        P.dbg = dbg ? (uint32_t)atoi(dbg) : 0;
    }
    grid = (uint32_t)((tiles + P.wt_per_block - 1) / P.wt_per_block);
    P.grid_main = grid;
    // per workgroup: at most 6 hashed updates per record, plus one cache flush per pass
    // (Net v2: two more updates per record and one more cache flush)
    P.mq_cap = P.wt_per_block * 64u * (PV_MQ_PER_REC + (c->net2_groups ? 2u : 0u)) + PV_CACHE_MAX * (c->net2_groups ? 3u : 2u);
    {
        const size_t need = (size_t)grid * P.mq_cap * 16;
        if (need > c->mq_bytes) {
            if (c->d_mq) hipFree(c->d_mq);
            if (c->d_tpbuf) hipFree(c->d_tpbuf);

            if (c->d_cb) hipFree(c->d_cb);
            c->d_mq = c->d_tpbuf = c->d_cb = nullptr;
            c->mq_bytes = 0;
            if (!hip_ok(e = hipMalloc(&c->d_mq, need)) || !hip_ok(e = hipMalloc(&c->d_tpbuf, need)) ||

                !hip_ok(e = hipMalloc(&c->d_cb, need)))
                return c->hipfail(e, "top-N update log");
            c->mq_bytes = need;
        }
    }
    if (grid > PV_MAX_GRID) return c->fail(PV_ECAPACITY, "grid of %u workgroups exceeds %d", grid, PV_MAX_GRID);
    if (P.mq_cap >= (1u << 24)) return c->fail(PV_ECAPACITY, "batch too large: %u update-log entries per workgroup", P.mq_cap);
    if (grid > c->cb_h_grid) {
        if (c->d_cb_h) hipFree(c->d_cb_h);
        c->d_cb_h = nullptr;
        c->cb_h_grid = 0;
        // run table: (2 << PV_MAX_REGIONS_LOG2) run keys x the grid padded to a multiple of 8
        if (!hip_ok(e = hipMalloc(&c->d_cb_h, (size_t)((grid + 7) & ~7u) << (PV_MAX_REGIONS_LOG2 + 4))))
            return c->hipfail(e, "region runs");
        c->cb_h_grid = grid;
    }
    P.mq = c->d_mq;
    P.mq_cnt = c->d_mq_cnt;
    P.reg_log2 = c->reg_log2;
    P.tab_live = c->d_tab_live;
    P.ovf = c->d_ovf;
    P.ovf_cnt = c->d_ovf_cnt;
    P.ovf_cap = c->ovf_cap;
    P.cb_run = (uint64_t *)c->d_cb_h;
    P.tp_hands = c->d_status + ST_HANDS;
    P.tp_buf = c->d_tpbuf;
    P.nn_cnt = c->d_status + ST_NNEW;
    P.nn = c->d_nn;
    P.nn_cap = c->nn_cap;
    P.iplog = c->d_iplog;
    P.iplog32 = c->d_iplog32;
    P.ipdir = c->d_ipdir;
    P.ipx_cnt = c->d_ipx_cnt;
    P.ipx_rep = c->d_ipx_rep;
    P.trash = c->d_trash;
    if ((uint64_t)grid * 4 > PV_TRASH_WAVES) return c->fail(PV_ECAPACITY, "grid of %u workgroups exceeds the trash area", grid);
    P.cb = c->d_cb;
    P.cb_cnt = c->d_cb_cnt;
    P.cb_hm = c->d_cb_cnt + 32768;
    {
        // grid ranges per combine workgroup (PV_CB_FAN, A/B runs): fewer, larger tables
        static const char *fan = getenv("PV_CB_FAN");
        P.cb_fan = fan ? std::max(1u, std::min(8u, (uint32_t)atoi(fan))) : c->cb_fan;
        while (P.cb_fan > 1 && (uint64_t)P.cb_fan * P.mq_cap >= (1u << 24)) P.cb_fan--; // run starts are 24-bit
        P.cb_grid = (grid + P.cb_fan - 1) / P.cb_fan;
    }
    P.stamps = c->d_stamps;
    P.dq = c->d_dq;
    P.dq_cnt = c->d_dq_cnt;
    // the specialised passes when nothing in the batch needs the general one: the lean pass
    // (one Net period, Ethernet, at most two IPv4 host subnets, a wave's tiles below 2^16 for
    // its packed lane counters), else the shift-free general pass. PV_NET_KERNEL=ns|general
    // forces one for A/B runs.
    static const char *force = getenv("PV_NET_KERNEL");
    // (every TCP packet for the exact LRU replay: the general pass emits them)
    const bool general = P.n_shift || P.net_filter_all || P.dbg || P.ndeep_net || c->tcp_exact_on() ||
                         (force && !strcmp(force, "general"));
    const uint32_t reg_grid = std::min<uint32_t>(grid, (uint32_t)(c->cus * c->reg_wg_per_cu));
    const uint64_t per_wave = ((uint64_t)P.wt_per_block / 4 + 1) * ((grid + reg_grid - 1) / reg_grid); // packed lane counters
    const bool lean = !general && P.linktype == 1 && P.nets.n4 <= 2 && P.skip_before == 0 && per_wave < 65535 &&
                      !(force && !strcmp(force, "ns"));
    // lean: the register-window pass (pv_net_kernel_reg, its top-IPs specialisation _tc), which
    // writes the compact IP log (4 B + a direction bit per record)
    P.ip_compact = lean ? 1u : 0u;
    P.ip_base = ((uint64_t)P.slot_of[0] << 60) | ((uint64_t)TM_IPV4 << 56) |
                ((uint64_t)((c->net_groups & PV_NET_CARDINALITY) ? 1 : 0) << 33);
    const bool tc = (c->net_groups & PV_NET_TOP_IPS) != 0;
    // PV_NET_KERNEL=span: the span-load pass (top-IPs groups), kept for A/B runs
    const bool span = lean && tc && force && !strcmp(force, "span");
    // both lean passes defer general-path records to pv_net_slow_list
    if (lean) {
        if (c->slow_cap < P.n) {
            if (c->d_slow) hipFree(c->d_slow);
            c->d_slow = nullptr;
            c->slow_cap = 0;
            if (!hip_ok(e = hipMalloc(&c->d_slow, (size_t)(P.n + PV_MAX_GRID) * 4))) return c->hipfail(e, "deferred record list");
            c->slow_cap = P.n;
        }
        P.slow_list = c->d_slow;
        P.slow_cnt = c->d_slow + c->slow_cap; // written for every range by the lean passes
    }
    *c->h_params = P;
    if (!hip_ok(e = fill_and_upload(c, c->d_params, c->h_params, sizeof P, st)))
        return c->hipfail(e, "parameter upload");
    c->net_kernel = general ? "pv_net_kernel"
                            : (lean ? (span ? "pv_net_kernel_span" : (tc ? "pv_net_kernel_reg_tc" : "pv_net_kernel_reg"))
                                    : "pv_net_kernel_ns");
    // pv_kernel_timing (bench roofline): the record-parse kernel alone, timed by the start and
    // end stamps of its own dispatch packet (hipExtLaunchKernelGGL), so no event marker packets
    // sit in the stream between the step's kernels
    const PvParams *dp = (const PvParams *)c->d_params;
    // (stamping a dispatch costs ~14 us of idle around it: only the batches pv_set_kernel_timing
    // asks for are stamped)
    const bool timed = c->timing_every && (c->timing_ctr++ % c->timing_every) == 0;
    hipEvent_t e0 = timed ? c->ev_start : nullptr, e1 = timed ? c->ev_stop : nullptr;
    if (general) hipExtLaunchKernelGGL(pv_net_kernel, dim3(grid), dim3(PV_NET_THREADS), 0, st, e0, e1, 0, dp);
    else if (lean) {
        // the lean pass, then its deferred general-path records (the dispatch stamps span both)
        if (span) hipExtLaunchKernelGGL(pv_net_kernel_span, dim3(reg_grid), dim3(PV_NET_THREADS), 0, st, e0, (hipEvent_t) nullptr, 0, dp);
        else if (tc) hipExtLaunchKernelGGL(pv_net_kernel_reg_tc, dim3(reg_grid), dim3(PV_NET_THREADS), 0, st, e0, (hipEvent_t) nullptr, 0, dp);
        else hipExtLaunchKernelGGL(pv_net_kernel_reg, dim3(reg_grid), dim3(PV_NET_THREADS), 0, st, e0, (hipEvent_t) nullptr, 0, dp);
        hipExtLaunchKernelGGL(pv_net_slow_list, dim3(c->cus * 2), dim3(256), 0, st, (hipEvent_t) nullptr, e1, 0, dp);
    }
    else hipExtLaunchKernelGGL(pv_net_kernel_ns, dim3(grid), dim3(PV_NET_THREADS), 0, st, e0, e1, 0, dp);
    e = hipGetLastError();
    if (e != hipSuccess) return c->hipfail(e, "launch pv_net_kernel");
    if (P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL))
        hipLaunchKernelGGL(pv_dns_suffix, dim3(grid), dim3(256), 0, st, (const PvParams *)c->d_params);
    // the DNS pass walks the logical grid's ranges with its resident grid
    const uint32_t dns_grid = std::min<uint32_t>(grid, (uint32_t)(c->cus * c->dns_wg_per_cu));
    if (P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL))
        hipLaunchKernelGGL(pv_dns_kernel_sfx, dim3(dns_grid), dim3(64 * PV_DNS_WAVES), 0, st, (const PvParams *)c->d_params);
    else if (P.f_flags)
        hipLaunchKernelGGL(pv_dns_kernel_f, dim3(dns_grid), dim3(64 * PV_DNS_WAVES), 0, st, (const PvParams *)c->d_params);
    else
        hipLaunchKernelGGL(pv_dns_kernel, dim3(dns_grid), dim3(64 * PV_DNS_WAVES), 0, st, (const PvParams *)c->d_params);
    if (c->net2_groups) hipLaunchKernelGGL(pv_net2_kernel, dim3(grid), dim3(256), 0, st, (const PvParams *)c->d_params);
    // top-N: combine each workgroup's updates into a list sorted by table region, merge
    // each region's runs in LDS, decode the names of new entries
    static int cb_threads = 0; // the kernel's own launch bound (tuning builds change it)
    if (!cb_threads) {
        hipFuncAttributes fa{};
        cb_threads = hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(pv_topn_combine)) == hipSuccess ? fa.maxThreadsPerBlock
                                                                                                             : PV_CB_THREADS;
    }
    hipLaunchKernelGGL(c->reg_log2 <= 10 ? pv_topn_combine : pv_topn_combine_r12, dim3(P.cb_grid), dim3(cb_threads), 0, st,
                       (const PvParams *)c->d_params);
    hipLaunchKernelGGL(pv_topn_merge, dim3(2u << c->reg_log2), dim3(pv_topn_merge_threads()), 0, st, (const PvParams *)c->d_params);
    // names: as many workgroups as are resident (LDS: two per CU), each pipelining its entries
    hipLaunchKernelGGL(pv_topn_names, dim3((uint32_t)c->cus * 2), dim3(256), 0, st, (const PvParams *)c->d_params);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch");

    // ---- transactions: pair responses with queries (sort by key, then record index)
    uint32_t status[ST_WORDS];
    HP(14);
    if (!hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "kernel execution");
    memcpy(status, c->h_status, sizeof status);
    c->dns_heavy = (uint64_t)status[ST_NDNS] * 2 > n;
    HP(4);
    {
        float ms = 0;
        if (timed && hipEventElapsedTime(&ms, c->ev_start, c->ev_stop) == hipSuccess) { c->kernel_ms += ms; c->kernel_launches++; }
    }
    // the parts this batch wrote are no longer clean
    // ---- DNS over TCP: the stage of a one-span batch (its segments came from the Net pass),
    // then this span's messages through the DNS pass, their events behind the UDP ones
    if (!c->tcp_pre) {
        if (int rc = tcp_stage(c, d_recs, d_offs, n, status[ST_TSEG], status[ST_TSEG_BYTES], first_sec, false, st)) return rc;
    }
    const uint32_t gt = tcp_pass(c, P, a, a + n, st, c->h_params + 1);
    if (gt) {
        // the TCP messages' events behind the UDP pass's key list
        if (P.want_events)
            hipLaunchKernelGGL(pv_xact_compact, dim3(gt), dim3(256), 0, st, (const PvParams *)c->d_params, grid,
                               status[ST_NKEYS]);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_dns_tcp");
        if (!hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "TCP DNS pass");
        memcpy(status, c->h_status, sizeof status);
    }
    for (uint32_t k = 0; k <= P.n_shift; k++) c->net.clean[P.slot_of[k]] = false;
    if (status[ST_NDNS] || gt)
        for (uint32_t k = 0; k <= P.n_dshift; k++) c->dns.clean[P.dslot_of[k]] = false;
    bool drained = false;
    if (int rc = drain_overflow(c, st, true, &drained)) return rc;
    uint32_t flags = status[ST_FLAGS];
    if (drained && !hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
    if (flags & PVF_ARENA_FULL) return c->fail(PV_ECAPACITY, "top-N name arena full");
    if (getenv("PV_TSTAMPS")) {
        // -DPV_TSTAMPS builds: mean cycles per workgroup of the top-N combine / merge phases
        std::vector<uint64_t> tv(65536 + (2u << c->reg_log2) * 8);
        if (hip_ok(hipMemcpy(tv.data(), c->d_stamps + (1u << 20), tv.size() * 8, hipMemcpyDeviceToHost))) {
            double cs[8] = {0}, ms[8] = {0};
            uint64_t nm = 0;
            for (uint32_t w = 0; w < grid; w++)
                for (int k = 0; k < 8; k++) cs[k] += (double)tv[w * 8 + k];
            for (uint32_t w = 0; w < (2u << c->reg_log2); w++) {
                const uint64_t *m = &tv[65536 + w * 8];
                if (!m[0] && !m[1]) continue;
                nm++;
                for (int k = 0; k < 8; k++) ms[k] += (double)m[k];
            }
            {
                // the ring Net pass's parsing waves (reg_grid x 4)
                std::vector<uint64_t> rv((size_t)reg_grid * (getenv("PV_RING_NP") ? atoi(getenv("PV_RING_NP")) : 4) * 8);
                if (hip_ok(hipMemcpy(rv.data(), c->d_stamps + (1u << 20) + 131072, rv.size() * 8, hipMemcpyDeviceToHost))) {
                    double a[8] = {0};
                    for (size_t w = 0; w < rv.size() / 8; w++)
                        for (int k = 0; k < 8; k++) a[k] += (double)rv[w * 8 + k];
                    const double nw = (double)(rv.size() / 8);
                    fprintf(stderr, "pv_tstamps ring parser (%u waves): wait_full=%.0f load_fields=%.0f dns_tcp_slow=%.0f hist=%.0f "
                                    "stores=%.0f loop=%.0f\n",
                            (unsigned)(rv.size() / 8), a[0] / nw, a[1] / nw, a[2] / nw, a[3] / nw, a[4] / nw, a[7] / nw);
                }
            }
            fprintf(stderr, "pv_tstamps combine (%u wg): init=%.0f insert=%.0f count=%.0f scan=%.0f out=%.0f | merge (%lu wg): "
                            "runs=%.0f load=%.0f insert=%.0f wb=%.0f names=%.0f\n",
                    grid, cs[0] / grid, cs[1] / grid, cs[2] / grid, cs[3] / grid, cs[4] / grid, (unsigned long)nm,
                    ms[0] / std::max<uint64_t>(nm, 1), ms[1] / std::max<uint64_t>(nm, 1), ms[2] / std::max<uint64_t>(nm, 1),
                    ms[3] / std::max<uint64_t>(nm, 1), ms[4] / std::max<uint64_t>(nm, 1));
            hipMemset(c->d_stamps + (1u << 20), 0, tv.size() * 8);
        }
    }
    if (getenv("PV_STAMPS")) {
        std::vector<uint64_t> stv((size_t)grid * 4 * 8);
        if (hip_ok(hipMemcpy(stv.data(), c->d_stamps, stv.size() * 8, hipMemcpyDeviceToHost))) {
            double sum[8] = {0};
            for (size_t w = 0; w < (size_t)grid * 4; w++)
                for (int k = 0; k < 8; k++) sum[k] += (double)stv[w * 8 + k];
            fprintf(stderr, "pv_stamps (mean cycles per wave, %u wave tiles/wg):", P.wt_per_block);
            static const char *nm[8] = {"slot", "commit", "barA", "issue", "parse", "lane", "barB", "flush"};
            for (int k = 0; k < 8; k++) fprintf(stderr, " %s=%.0f", nm[k], sum[k] / (grid * 4.0));
            fprintf(stderr, "\n");
        }
    }
    HP(5);
    if (int rc = pair_stage(c, P, status[ST_NEV], status[ST_NKEYS], status[ST_NRESP], n, st,
                            (uint64_t)(grid + gt) * P.wt_per_block * 64u))
        return rc;
    HP(6);
    // top_slow updates of the transaction stage (only when it ran)
    if ((status[ST_NEV] || c->n_pend) && P.want_events)
        if (int rc = drain_overflow(c, st)) return rc;

    // ---- window bookkeeping (host mirror of each manager's _period_shift)
    for (const Shift &sh : nsh) win_shift(c, c->net, sh.sec);
    for (const Shift &sh : dsh) {
        win_shift(c, c->dns, sh.sec);
        c->dns_shifts.emplace_back(sh.sec, c->dns.slot_at(0));
        c->dns_shift_ord.emplace_back(sh.sec, c->dns.ordinal);
    }
    c->records_seen += n;
    const int prc = purge_tables(c, st);
    HP(7);
    return prc;
}

// Both managers' shifts of a batch (Net from the record seconds, DNS from the prescan bits
// and the TCP messages). A batch that may shift DNS windows, or that the Net shifts split
// into spans, runs its TCP stage here, ahead of the spans (the prescan emits the segments);
// any other batch runs it inside its one span, behind the Net pass (c->tcp_pre).
int batch_shifts(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                 const uint32_t *sc_idx, const uint32_t *sc_sec, hipStream_t st, std::vector<Shift> &nsh,
                 std::vector<Shift> &dsh)
{
    c->tcp_pre = false;
    c->tcp_nmsg = 0;
    c->tcp_ords.clear();
    c->tcp_items.clear();
    // the batch's latest second (its last record's, unless the timestamps go back somewhere)
    int64_t top = info->last_sec;
    if (!info->monotone)
        for (uint32_t k = 0; k < info->n_sec_changes; k++) top = std::max<int64_t>(top, (int64_t)sc_sec[k]);
    if (c->sample_rate < 100) {
        // deep sampling draws per DNS event in stream order, DNS-over-TCP messages among them:
        // the TCP stage runs ahead of the spans so their order is known first
        c->tcp_pre = true;
        uint32_t tseg[2] = {0, 0};
        if (int rc = dns_prescan(c, d_recs, d_offs, info->n_records, st, true, tseg)) return rc;
        const bool dns_may = c->cfg.num_periods > 1 && top >= c->dns.next_shift_sec;
        c->eoc_stage = c->eoc_batch;
        if (int rc = tcp_stage(c, d_recs, d_offs, info->n_records, tseg[0], tseg[1], (uint32_t)info->first_sec, true, st))
            return rc;
        if (c->cfg.num_periods <= 1) return 0;
        const bool net_may = top >= c->net.next_shift_sec;
        if (!net_may && !dns_may) return 0;
        if (net_may) net_shifts_of(c->net.next_shift_sec, info, sc_idx, sc_sec, nsh);
        if (dns_may) dns_shifts_of(c->dns.next_shift_sec, c->h_dbits, info->n_records, info, sc_idx, sc_sec, c->tcp_ords, dsh);
        return 0;
    }
    if (c->cfg.num_periods <= 1) return 0;
    const bool net_may = top >= c->net.next_shift_sec, dns_may = top >= c->dns.next_shift_sec;
    if (!net_may && !dns_may) return 0;
    if (net_may) net_shifts_of(c->net.next_shift_sec, info, sc_idx, sc_sec, nsh);
    c->tcp_pre = dns_may || nsh.size() > PV_MAX_SHIFTS;
    if (c->tcp_pre) {
        uint32_t tseg[2] = {0, 0};
        if (int rc = dns_prescan(c, d_recs, d_offs, info->n_records, st, true, tseg)) return rc;
        c->eoc_stage = c->eoc_batch;
        if (int rc = tcp_stage(c, d_recs, d_offs, info->n_records, tseg[0], tseg[1], (uint32_t)info->first_sec, dns_may, st))
            return rc;
    }
    if (dns_may) dns_shifts_of(c->dns.next_shift_sec, c->h_dbits, info->n_records, info, sc_idx, sc_sec, c->tcp_ords, dsh);
    return 0;
}

} // namespace

int x_grow_dev(pv_ctx *c, void **p, size_t &have, size_t need, const char *what)
{
    if (need <= have) return 0;
    hipError_t e;
    if (*p) hipFree(*p);
    *p = nullptr;
    have = 0;
    if (!hip_ok(e = hipMalloc(p, std::max<size_t>(need, 256)))) return c->hipfail(e, what);
    have = std::max<size_t>(need, 256);
    return 0;
}
// The BPF filter on a device batch: keep flags and sizes (pv_bpf_keep), their exclusive scans (byte
// offsets, ranks), the kept records compacted into d_frecs / d_foffs (pv_bpf_gather), and the
// kept run's index info and ts_sec change points (pv_bpf_secs). The caller holds c->mu.
int bpf_filter_device(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info, hipStream_t st,
                      pv_index_info &out, std::vector<uint32_t> &sci, std::vector<uint32_t> &scs)
{
    hipError_t e;
    const uint32_t n = (uint32_t)info->n_records;
    memset(&out, 0, sizeof out);
    if (c->bpf_dirty || !c->d_bpf) {
        if (c->d_bpf) hipFree(c->d_bpf);
        c->d_bpf = nullptr;
        if (!hip_ok(e = hipMalloc(&c->d_bpf, c->bpf.size() * sizeof(pv_bpf_insn))) ||
            !hip_ok(e = hipMemcpy(c->d_bpf, c->bpf.data(), c->bpf.size() * sizeof(pv_bpf_insn), hipMemcpyHostToDevice)))
            return c->hipfail(e, "BPF program");
        c->d_bpf_n = c->bpf.size();
        c->bpf_dirty = false;
    }
    if (n > c->fwork_n) {
        for (void *p : {(void *)c->d_fwork, (void *)c->d_foffs, (void *)c->d_fsc}) if (p) hipFree(p);
        c->d_fwork = c->d_foffs = c->d_fsc = nullptr;
        c->fwork_n = 0;
        if (!hip_ok(e = hipMalloc(&c->d_fwork, (size_t)n * 16)) || !hip_ok(e = hipMalloc(&c->d_foffs, (size_t)n * 4)) ||
            !hip_ok(e = hipMalloc(&c->d_fsc, (size_t)n * 8 + 64)))
            return c->hipfail(e, "BPF filter buffers");
        c->fwork_n = n;
    }
    if (info->bytes_used + PV_RECS_PAD > c->frecs_bytes) {
        if (c->d_frecs) hipFree(c->d_frecs);
        c->d_frecs = nullptr;
        c->frecs_bytes = 0;
        if (!hip_ok(e = hipMalloc(&c->d_frecs, info->bytes_used + PV_RECS_PAD)) ||
            !hip_ok(e = hipMemsetAsync(c->d_frecs, 0, info->bytes_used + PV_RECS_PAD, st)))
            return c->hipfail(e, "BPF filter buffers");
        c->frecs_bytes = info->bytes_used + PV_RECS_PAD;
    }
    size_t tb = 0;
    if (!hip_ok(e = pv_exclusive_scan_u32(nullptr, &tb, nullptr, nullptr, n, st))) return c->hipfail(e, "scan size");
    if (int rc = x_grow_dev(c, &c->d_fscan, c->fscan_bytes, tb, "BPF scan")) return rc;
    uint32_t *sz = c->d_fwork, *kf = sz + n, *boff = kf + n, *rank = boff + n;
    const uint32_t grid = (n + 255) / 256;
    hipLaunchKernelGGL(pv_bpf_keep, dim3(grid), dim3(256), 0, st, d_recs, d_offs, n, (const PvBpfIns *)c->d_bpf,
                       (uint32_t)c->d_bpf_n, sz, kf);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_bpf_keep");
    tb = c->fscan_bytes;
    if (!hip_ok(e = pv_exclusive_scan_u32(c->d_fscan, &tb, sz, boff, n, st))) return c->hipfail(e, "scan");
    tb = c->fscan_bytes;
    if (!hip_ok(e = pv_exclusive_scan_u32(c->d_fscan, &tb, kf, rank, n, st))) return c->hipfail(e, "scan");
    uint32_t tail[4];
    if (!hip_ok(e = hipMemcpyAsync(&tail[0], boff + n - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&tail[1], sz + n - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&tail[2], rank + n - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&tail[3], kf + n - 1, 4, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "BPF filter");
    const uint64_t bytes = (uint64_t)tail[0] + tail[1];
    const uint32_t nk = tail[2] + tail[3];
    if (!nk) return 0;
    hipLaunchKernelGGL(pv_bpf_gather, dim3(grid), dim3(256), 0, st, d_recs, d_offs, n, (const uint32_t *)sz, (const uint32_t *)boff,
                       (const uint32_t *)rank, c->d_frecs, c->d_foffs);
    // the kept run's change points (sz / kf / boff reused: flags, seconds, positions)
    uint32_t *flag = sz, *sec = kf, *pos = boff, *down = c->d_fsc + 2 * (size_t)n;
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemsetAsync(down, 0, 4, st))) return c->hipfail(e, "BPF filter");
    hipLaunchKernelGGL(pv_bpf_secs, dim3((nk + 255) / 256), dim3(256), 0, st, (const uint8_t *)c->d_frecs, (const uint32_t *)c->d_foffs,
                       nk, flag, sec, down);
    tb = c->fscan_bytes;
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = pv_exclusive_scan_u32(c->d_fscan, &tb, flag, pos, nk, st)))
        return c->hipfail(e, "BPF filter");
    hipLaunchKernelGGL(pv_bpf_secs_compact, dim3((nk + 255) / 256), dim3(256), 0, st, (const uint32_t *)flag, (const uint32_t *)pos,
                       (const uint32_t *)sec, nk, n, c->d_fsc, c->d_fsc + n);
    uint32_t w[4], lo = 0, hi_off = 0;
    uint32_t h0[4], h1[4];
    if (!hip_ok(e = hipGetLastError()) ||
        !hip_ok(e = hipMemcpyAsync(&w[0], pos + nk - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&w[1], flag + nk - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&w[2], down, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&hi_off, c->d_foffs + nk - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(h0, c->d_frecs, 16, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)) ||
        !hip_ok(e = hipMemcpy(h1, c->d_frecs + hi_off, 16, hipMemcpyDeviceToHost)))
        return c->hipfail(e, "BPF filter");
    (void)lo;
    const uint32_t nch = w[0] + w[1];
    sci.resize(nch);
    scs.resize(nch);
    if (nch && (!hip_ok(e = hipMemcpy(sci.data(), c->d_fsc, (size_t)nch * 4, hipMemcpyDeviceToHost)) ||
                !hip_ok(e = hipMemcpy(scs.data(), c->d_fsc + n, (size_t)nch * 4, hipMemcpyDeviceToHost))))
        return c->hipfail(e, "BPF filter");
    out.n_records = nk;
    out.bytes_used = bytes;
    out.first_sec = h0[0];
    out.first_nsec = c->cfg.ts_nano ? (int64_t)h0[1] : (int64_t)h0[1] * 1000;
    out.last_sec = h1[0];
    out.last_nsec = c->cfg.ts_nano ? (int64_t)h1[1] : (int64_t)h1[1] * 1000;
    out.monotone = w[2] == 0;
    out.n_sec_changes = nch;
    return 0;
}

int pv_process_device(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                      const uint32_t *sc_idx, const uint32_t *sc_sec, void *stream)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = merged_refuse(c)) return rc;
    hipSetDevice(c->device);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    hipStream_t saved = c->stream;
    c->stream = st;
    struct Restore { pv_ctx *c; hipStream_t s; ~Restore() { c->stream = s; } } restore{c, saved};
    // the end of the capture (pv_set_end_of_capture): a direct call is the capture's final batch;
    // pv_process_host's ingest loops mark their final batch themselves
    if (!c->in_host) c->eoc_batch = c->eoc_armed;
    struct EocDone {
        pv_ctx *c;
        ~EocDone()
        {
            c->eoc_stage = false;
            if (!c->in_host) c->eoc_armed = c->eoc_batch = false;
        }
    } eoc_done{c};
    if (info->n_records == 0) return 0;
    if (info->n_records > c->max_records) return c->fail(PV_ECAPACITY, "batch of %llu records exceeds max_records %llu",
                                           (unsigned long long)info->n_records, (unsigned long long)c->max_records);
    pv_index_info finfo;
    std::vector<uint32_t> fsci, fscs;
    if (!c->bpf.empty()) {
        // the pcap input's BPF filter (PcapInputStream.cpp:485-488) over the batch in HBM: the kept
        // records become the batch
        if (int rc = bpf_filter_device(c, d_recs, d_offs, info, st, finfo, fsci, fscs)) return rc;
        if (finfo.n_records == 0) return 0;
        d_recs = c->d_frecs;
        d_offs = c->d_foffs;
        info = &finfo;
        sc_idx = fsci.data();
        sc_sec = fscs.data();
    }
    const uint64_t n = info->n_records;
    ensure_started(c, info->first_sec, info->first_nsec);
    std::vector<Shift> nsh, dsh;
    if (int rc = batch_shifts(c, d_recs, d_offs, info, sc_idx, sc_sec, st, nsh, dsh)) return rc;
    HP(3);
    // spans of at most PV_MAX_SHIFTS shifts of each manager, cut at the shifting record
    uint64_t a = 0;
    size_t ni = 0, di = 0;
    while (a < n) {
        uint64_t b = n;
        if (nsh.size() - ni > PV_MAX_SHIFTS) b = std::min<uint64_t>(b, nsh[ni + PV_MAX_SHIFTS].idx);
        if (dsh.size() - di > PV_MAX_SHIFTS) b = std::min<uint64_t>(b, dsh[di + PV_MAX_SHIFTS].idx);
        std::vector<Shift> ns, ds;
        for (; ni < nsh.size() && nsh[ni].idx < b; ni++) ns.push_back({nsh[ni].sec, nsh[ni].idx - a, 0});
        for (; di < dsh.size() && dsh[di].idx < b; di++) ds.push_back({dsh[di].sec, dsh[di].idx - a, dsh[di].ord - 4 * a});
        uint64_t rec_bytes = info->bytes_used;
        if (b < n) {
            uint32_t ob = 0;
            hipError_t e;
            if (!hip_ok(e = hipMemcpyAsync(&ob, d_offs + b, 4, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
                return c->hipfail(e, "span end");
            rec_bytes = ob;
        }
        // (a batch with a TCP stage ahead of its spans ran it in batch_shifts)
        c->eoc_stage = c->eoc_batch && b == n && !c->tcp_pre;
        if (int rc = process_span(c, d_recs, d_offs, a, b - a, rec_bytes, ns, ds, (uint32_t)info->first_sec, st)) return rc;
        a = b;
    }
    c->last_sec = info->last_sec;
    c->last_nsec = info->last_nsec;
    return 0;
}

int pv_synchronize(pv_ctx *c)
{
    flush_fills(c);
    hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    return 0;
}

namespace {

int ingest_setup(pv_ctx *c)
{
    if (c->copy_stream) return 0;
    hipError_t e;
    // 128 MiB pieces: the top-N merge's cost per batch is per region, not per entry, so larger
    // pieces amortise it (C5 100M: 172.5 / 184.2 / 184.9 Mpkt/s at 64 / 128 / 256 MiB,
    // profiles/r5/c5_chunk*.log)
    size_t chunk = 128ull << 20;
    if (const char *v = getenv("PV_INGEST_CHUNK_MB")) chunk = std::max<size_t>(1, strtoull(v, nullptr, 10)) << 20;
    c->stage_recs = std::min<uint64_t>(c->max_records, chunk / 16 + 1);
    c->stage_bytes = chunk;
    if (const char *v = getenv("PV_INGEST_RING")) c->ring_n = (uint32_t)std::min<unsigned long>(8, std::max<unsigned long>(3, strtoul(v, nullptr, 10)));
    c->pool.reset(new pvi::Pool(pvi::default_threads()));
    if (!hip_ok(e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking))) return c->hipfail(e, "copy stream");
    for (auto &st : c->stage) {
        if (!hip_ok(e = hipHostMalloc((void **)&st.h_recs, chunk + PV_RECS_PAD, hipHostMallocDefault)) ||
            !hip_ok(e = hipHostMalloc((void **)&st.h_offs, c->stage_recs * 4, hipHostMallocDefault)) ||
            !hip_ok(e = hipMalloc(&st.d_recs, chunk + PV_RECS_PAD)) || !hip_ok(e = hipMalloc(&st.d_offs, c->stage_recs * 4)) ||
            !hip_ok(e = hipEventCreateWithFlags(&st.copied, hipEventDisableTiming)))
            return c->hipfail(e, "ingest staging");
        st.sci.resize(1 << 16);
        st.scs.resize(1 << 16);
        // device record index state for a chunk of up to `chunk` bytes
        const uint32_t nseg = (uint32_t)((2 * chunk + PV_IX_SEG - 1) / PV_IX_SEG); // a ring run: tail + chunk
        const size_t bytes = 256 + (size_t)nseg * 8 * 3 + (size_t)(nseg + 1) * 4 * 2 + 64 + st.sci.size() * 8 + 1024;
        if (!hip_ok(e = hipMalloc(&st.d_ix, bytes)) ||
            !hip_ok(e = hipHostMalloc((void **)&st.h_ix, 256 + 64 + st.sci.size() * 8 + 1024, hipHostMallocDefault)))
            return c->hipfail(e, "device index state");
        st.ix_nseg = nseg;
    }
    if (const char *v = getenv("PV_INGEST_INDEX")) c->device_index = strcmp(v, "host") != 0;
    return 0;
}

// The record index of the records at [first, end) of d_base (256-B aligned, first < 256),
// already on the device, on the device (pv_index.hip): offsets (relative to d_base) into
// d_offs, the ts_sec change points into st.sci / st.scs (sorted), st.info as pv_index_records
// fills it (bytes_used relative to d_base), *capped when more complete records follow the
// first stage_recs. `hfirst` is byte `first` in host memory (headers of the first and last
// records). Returns 1 when the validation passes do not settle (adversarial bytes: the caller
// walks the block on the host), < 0 on an error.
int device_index(pv_ctx *c, pv_ctx::Stage &st, const uint8_t *d_base, uint32_t first, const uint8_t *hfirst, size_t L,
                 uint32_t *d_offs, hipStream_t s, bool *capped)
{
    const uint32_t nseg = (uint32_t)((L + PV_IX_SEG - 1) / PV_IX_SEG);
    if (nseg > st.ix_nseg) return c->fail(PV_ECAPACITY, "index block of %zu bytes exceeds the index state", L);
    *capped = false;
    uint8_t *d = st.d_ix;
    PvIxParams X;
    memset(&X, 0, sizeof X);
    size_t at = 256;
    auto take = [&](size_t b) { uint8_t *q = d + at; at += (b + 63) & ~(size_t)63; return q; };
    X.recs = d_base;
    X.bytes = L;
    X.first = first;
    X.nseg = nseg;
    X.frac_lim = c->cfg.ts_nano ? 1000000000u : 1000000u;
    memcpy(&X.sec0, hfirst, 4);
    X.start = (uint64_t *)take((size_t)nseg * 8);
    X.exit[0] = (uint64_t *)take((size_t)nseg * 8);
    X.exit[1] = (uint64_t *)take((size_t)nseg * 8);
    X.cnt = (uint32_t *)take((size_t)nseg * 4);
    X.base = (uint32_t *)take((size_t)(nseg + 1) * 4);
    X.status = (uint32_t *)take(32);
    X.sci = (uint32_t *)take(st.sci.size() * 4);
    X.scs = (uint32_t *)take(st.sci.size() * 4);
    X.offs = d_offs;
    X.max_records = c->stage_recs;
    X.max_changes = (uint32_t)st.sci.size();
    uint32_t *h = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(st.h_ix) + 256); // read-back words
    *st.h_ix = X;
    const PvIxParams *dX = reinterpret_cast<const PvIxParams *>(d);
    const dim3 g((nseg + 255) / 256), b(256);
    hipError_t e;
    if (!hip_ok(e = hipMemcpyAsync(d, st.h_ix, sizeof X, hipMemcpyHostToDevice, s)) ||
        !hip_ok(e = hipMemsetAsync(X.status, 0, 32, s)))
        return c->hipfail(e, "device index");
    hipLaunchKernelGGL(pv_ix_guess, dim3((nseg + 3) / 4), dim3(256), 0, s, dX); // a wave per segment
    // one validation pass, then the scan, the offsets, the change points and the last change's
    // neighbours, read back under one synchronisation: a pass that changed nothing (the guesses
    // were right) settles the chain. Otherwise the passes run on, one read-back each, until they
    // settle, and the rest runs again (its first run only wrote offsets of valid walks).
    const uint32_t pre = 1024; // change points read back with the status; more in a second copy
    const uint32_t secs_grid = (uint32_t)std::min<uint64_t>((c->stage_recs + 255) / 256, (uint64_t)c->cus * 8);
    uint32_t src = 0;
    auto fix_pass = [&]() {
        hipMemsetAsync(X.status, 0, 4, s);
        hipLaunchKernelGGL(pv_ix_fix, g, b, 0, s, dX, src);
        src ^= 1;
    };
    auto rest = [&]() -> hipError_t {
        hipLaunchKernelGGL(pv_ix_scan, dim3(1), dim3(1024), 0, s, dX);
        hipMemsetAsync(X.status + 1, 0, 28, s);
        hipLaunchKernelGGL(pv_ix_write, g, b, 0, s, dX);
        hipLaunchKernelGGL(pv_ix_secs, dim3(std::max(1u, secs_grid)), dim3(256), 0, s, dX, (uint32_t)c->stage_recs);
        hipLaunchKernelGGL(pv_ix_cut, dim3(1), dim3(64), 0, s, dX);
        hipError_t e2 = hipGetLastError();
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h, X.status, 32, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 8, X.base + nseg, 4, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 10, X.exit[src] + nseg - 1, 8, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 16, X.sci, pre * 4, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 16 + st.sci.size(), X.scs, pre * 4, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipStreamSynchronize(s);
        return e2;
    };
    fix_pass();
    if (!hip_ok(e = rest())) return c->hipfail(e, "device index");
    if (h[0] != 0) {
        bool settled = false;
        for (int pass = 1; pass < 64 && !settled; pass++) {
            fix_pass();
            if (!hip_ok(e = hipMemcpyAsync(h, X.status, 4, hipMemcpyDeviceToHost, s)) || !hip_ok(e = hipStreamSynchronize(s)))
                return c->hipfail(e, "device index pass");
            settled = h[0] == 0;
        }
        if (!settled) return 1;
        if (!hip_ok(e = rest())) return c->hipfail(e, "device index");
    }
    const uint64_t total = h[8];
    uint64_t chain_end = 0;
    memcpy(&chain_end, h + 10, 8);
    const uint64_t n = std::min<uint64_t>(total, c->stage_recs);
    pv_index_info &info = st.info;
    memset(&info, 0, sizeof info);
    info.monotone = 1;
    info.n_records = n;
    info.bytes_used = chain_end & ~PV_IX_STOP;
    if (n == 0) return 0;
    const uint32_t nc = h[1];
    const uint32_t last_off = h[3];
    st.cut_o[0] = h[5];
    st.cut_o[1] = h[6];
    if (nc > st.sci.size()) return c->fail(PV_ECAPACITY, "more than %zu ts_sec changes in one ingest chunk", st.sci.size());
    if (nc > pre &&
        (!hip_ok(e = hipMemcpyAsync(h + 16, X.sci, (size_t)nc * 4, hipMemcpyDeviceToHost, s)) ||
         !hip_ok(e = hipMemcpyAsync(h + 16 + st.sci.size(), X.scs, (size_t)nc * 4, hipMemcpyDeviceToHost, s)) ||
         !hip_ok(e = hipStreamSynchronize(s))))
        return c->hipfail(e, "device index change points");
    std::vector<std::pair<uint32_t, uint32_t>> ch(nc);
    for (uint32_t k = 0; k < nc; k++) ch[k] = {h[16 + k], h[16 + st.sci.size() + k]};
    std::sort(ch.begin(), ch.end());
    for (uint32_t k = 0; k < nc; k++) { st.sci[k] = ch[k].first; st.scs[k] = ch[k].second; }
    info.n_sec_changes = nc;
    info.monotone = h[2] ? 0 : 1;
    uint32_t h0[4], h1[4];
    memcpy(h0, hfirst, 16);
    memcpy(h1, hfirst + (last_off - first), 16);
    if (n < total) {
        info.bytes_used = (uint64_t)last_off + 16 + h1[2];
        *capped = true;
    }
    info.first_sec = h0[0];
    info.first_nsec = c->cfg.ts_nano ? (int64_t)h0[1] : (int64_t)h0[1] * 1000;
    info.last_sec = h1[0];
    info.last_nsec = c->cfg.ts_nano ? (int64_t)h1[1] : (int64_t)h1[1] * 1000;
    return 0;
}

// device_index's fallback: the host walk of the block, its offsets copied to d_offs
int host_index_run(pv_ctx *c, pv_ctx::Stage &st, const uint8_t *d_base, uint32_t first, const uint8_t *hfirst, size_t end,
                   uint32_t *d_offs, bool *capped)
{
    (void)d_base;
    pv_index_info &info = st.info;
    if (int rc = pv_index_records(hfirst, end - first, c->cfg.ts_nano, st.h_offs, c->stage_recs, st.sci.data(), st.scs.data(),
                                  (uint32_t)st.sci.size(), &info))
        return c->fail(rc, "record index failed");
    const uint64_t n = info.n_records;
    *capped = false;
    if (n == c->stage_recs && info.bytes_used + 16 <= end - first) {
        uint32_t cl;
        memcpy(&cl, hfirst + info.bytes_used + 8, 4);
        *capped = info.bytes_used + 16 + (uint64_t)cl <= end - first;
    }
    for (uint64_t i = 0; i < n; i++) st.h_offs[i] += first;
    info.bytes_used += first;
    if (info.n_sec_changes > 1 && info.n_sec_changes <= st.sci.size()) {
        const uint32_t cut = st.sci[info.n_sec_changes - 1];
        st.cut_o[0] = st.h_offs[cut - 1];
        st.cut_o[1] = st.h_offs[cut];
    }
    hipError_t e;
    if (n && (!hip_ok(e = hipMemcpyAsync(d_offs, st.h_offs, n * 4, hipMemcpyHostToDevice, c->stream)) ||
              !hip_ok(e = hipStreamSynchronize(c->stream))))
        return c->hipfail(e, "H2D offsets");
    return 0;
}

bool host_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}


double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

} // namespace

// pv_dns_event_seconds over records in host memory, through the ingest staging (chunked).
static int dns_event_seconds_batch(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                                   const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n);
int pv_dns_event_seconds_host(pv_ctx *c, const uint8_t *recs, size_t bytes, int64_t *secs, uint32_t max, uint32_t *n)
{
    hipSetDevice(c->device);
    *n = 0;
    c->plan_draws = 0;
    if (c->tcp_active) return c->fail(PV_EINVAL, "pv_dns_event_seconds_host after DNS-over-TCP state (call it before the first batch)");
    struct TcpClean { pv_ctx *c; ~TcpClean() { std::lock_guard<std::mutex> g(c->mu); tcp_reset(c); } } clean{c};
    if (int rc = ingest_setup(c)) return rc;
    pv_ctx::Stage &st = c->stage[0];
    size_t pos = 0;
    uint32_t k = 0;
    while (pos < bytes) {
        const size_t L = std::min(c->stage_bytes, bytes - pos);
        int rc = pvi::index_records_parallel(*c->pool, recs + pos, L, c->cfg.ts_nano, st.h_offs, c->stage_recs,
                                             st.sci.data(), st.scs.data(), (uint32_t)st.sci.size(), &st.info, st.h_recs);
        if (rc) return c->fail(rc, "record index failed");
        if (st.info.n_records == 0) return c->fail(PV_ECAPACITY, "record larger than the ingest chunk");
        const size_t used = st.info.bytes_used;
        hipError_t e;
        if (!hip_ok(e = hipMemcpyAsync(st.d_recs, st.h_recs, used, hipMemcpyHostToDevice, c->stream)) ||
            !hip_ok(e = hipMemsetAsync(st.d_recs + used, 0, PV_RECS_PAD, c->stream)) ||
            !hip_ok(e = hipMemcpyAsync(st.d_offs, st.h_offs, st.info.n_records * 4, hipMemcpyHostToDevice, c->stream)))
            return c->hipfail(e, "H2D");
        std::vector<int64_t> part(st.info.n_records + 1);
        uint32_t m = 0;
        {
            std::lock_guard<std::mutex> g(c->mu);
            if ((rc = dns_event_seconds_batch(c, st.d_recs, st.d_offs, &st.info, st.sci.data(), st.scs.data(), part.data(),
                                              (uint32_t)part.size(), &m)))
                return rc;
        }
        for (uint32_t j = 0; j < m; j++) {
            if (k && secs[k - 1] == part[j]) continue; // a second split across chunks
            if (k >= max) return c->fail(PV_ECAPACITY, "more than %u DNS seconds", max);
            secs[k++] = part[j];
        }
        pos += used;
    }
    *n = k;
    return 0;
}

// dnstap input (DnstapInputStream, src/inputs/dnstap/DnstapInputStream.cpp:33-92) into the Net
// and DNS handlers' process_dnstap paths (net/v1 NetStreamHandler.cpp:549-620,832-843;
// dns/v1 DnsStreamHandler.cpp:260-266,839-909,1376-1412). The host decodes the Frame Streams
// file (pv_dnstap.cpp) and lays each event out as a PvDtEv plus a linktype-101 record (IP
// header with the query / response addresses, UDP header, the DNS message); the managers'
// period shifts are applied between spans of events; pv_dnstap_kernel does the accounting.
int dns_period_shift(pv_ctx *c, int64_t sec, int64_t nsec);
// lib::utils::match_subnet(IPv4subnetList &, IPv6subnetList &, const std::string &) as the
// dnstap proxy calls it (libs/visor_utils/utils.cpp:26-80): the std::string is the message's raw
// address bytes, which pcpp::IPv4Address / IPv6Address parse as TEXT (inet_pton on the string up
// to its first NUL; an unparsable one is the unspecified address, which isValid() rejects), so a
// 4- or 16-byte binary address practically never matches
static bool dt_match_subnet(const pv_ctx *c, const std::vector<uint8_t> &raw)
{
    const std::string txt(raw.begin(), std::find(raw.begin(), raw.end(), (uint8_t)0));
    in_addr a4{};
    if (inet_pton(AF_INET, txt.c_str(), &a4) == 1 && a4.s_addr != 0) {
        for (auto &n : c->dt_v4) {
            if (n.second == 0) return true;
            const uint32_t mask = htonl(0xFFFFFFFFu << (32 - n.second));
            if (((a4.s_addr ^ n.first) & mask) == 0) return true;
        }
        return false;
    }
    uint8_t a6[16] = {0};
    static const uint8_t zero[16] = {0};
    if (inet_pton(AF_INET6, txt.c_str(), a6) == 1 && memcmp(a6, zero, 16) != 0) {
        for (auto &n : c->dt_v6) {
            const uint32_t bytes = n.second / 8, bits = n.second % 8;
            bool r = false;
            if (bytes > 0) r = memcmp(n.first.data(), a6, bytes) == 0;
            if ((r || n.second < 8) && bits > 0) r = (n.first[bytes] >> (8 - bits)) == (a6[bytes] >> (8 - bits));
            if (r) return true;
        }
    }
    return false;
}

int pv_set_dnstap_only_hosts(pv_ctx *c, const char *hosts)
{
    if (!c) return PV_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (!hosts) {
        c->dt_v4.clear();
        c->dt_v6.clear();
        c->dt_only_hosts = false;
        return 0;
    }
    // parse_host_specs (libs/visor_utils/utils.cpp:128-164), its error texts. The lists are
    // parsed into locals and committed together with the flag only when every spec parses: a
    // failing call leaves the previous filter as it was (the reference throws from the input
    // proxy's constructor, so no half-applied filter ever exists)
    decltype(c->dt_v4) v4;
    decltype(c->dt_v6) v6;
    const std::string s = hosts;
    size_t pos = 0;
    while (pos < s.size()) {
        const size_t e = s.find(',', pos);
        const std::string host = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
        pos = e == std::string::npos ? s.size() : e + 1;
        if (host.empty()) continue;
        const size_t d = host.find('/');
        if (d == std::string::npos) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        const std::string ip = host.substr(0, d), cs = host.substr(d + 1);
        if (cs.empty() || !std::all_of(cs.begin(), cs.end(), ::isdigit)) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        const int cidr = atoi(cs.c_str());
        if (ip.find(':') != std::string::npos) {
            std::array<uint8_t, 16> a{};
            if (cidr < 0 || cidr > 128) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (inet_pton(AF_INET6, ip.c_str(), a.data()) != 1) return c->fail(PV_EINVAL, "invalid IPv6 address: %s", ip.c_str());
            v6.push_back({a, (uint32_t)cidr});
        } else {
            in_addr a{};
            if (cidr < 0 || cidr > 32) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (inet_pton(AF_INET, ip.c_str(), &a) != 1) return c->fail(PV_EINVAL, "invalid IPv4 address: %s", ip.c_str());
            v4.push_back({a.s_addr, (uint32_t)cidr});
        }
    }
    c->dt_v4 = std::move(v4);
    c->dt_v6 = std::move(v6);
    c->dt_only_hosts = true;
    return 0;
}

int pv_process_dnstap(pv_ctx *c, const uint8_t *buf, size_t bytes, uint32_t msg_type_mask)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = merged_refuse(c)) return rc;
    hipSetDevice(c->device);
    std::vector<pvi::DtMessage> msgs;
    uint32_t frames = 0;
    pvi::dnstap_decode(buf, bytes, msgs, &frames);
    if (c->dt_only_hosts) {
        // DnstapInputEventProxy::dnstap_cb's only_hosts block, in its branch order: both addresses
        // and neither matches, one address that does not match, and (its final else) every
        // other message: filtered before any handler sees it
        std::vector<pvi::DtMessage> kept;
        for (auto &m : msgs) {
            bool filt;
            if (m.has_qaddr && m.has_raddr) filt = !dt_match_subnet(c, m.qaddr) && !dt_match_subnet(c, m.raddr);
            else if (m.has_qaddr && !dt_match_subnet(c, m.qaddr)) filt = true;
            else if (m.has_raddr && !dt_match_subnet(c, m.raddr)) filt = true;
            else filt = true;
            if (!filt) kept.push_back(std::move(m));
        }
        msgs.swap(kept);
    }
    const size_t n = msgs.size();
    if (n == 0) return 0;
    if (n > 0x3fffffffull) return c->fail(PV_ECAPACITY, "too many dnstap events in one call");
    std::vector<PvDtEv> ev(n);
    std::vector<uint32_t> offs(n);
    std::vector<int64_t> ssec(n), snsec(n);
    std::vector<uint8_t> arena;
    arena.reserve(n * 96 + bytes);
    timespec now{};
    for (size_t j = 0; j < n; j++) {
        const pvi::DtMessage &m = msgs[j];
        PvDtEv &e = ev[j];
        memset(&e, 0, sizeof e);
        const uint32_t t = m.type;
        // the event's timestamp (DnsMetricsManager::process_dnstap :1379-1402): the response
        // time for CLIENT/AUTH/RESOLVER responses, the query time for their queries, else now
        // (also when that time is absent, where the reference leaves the stamp unset)
        int64_t sec = -1, nsec = 0;
        if ((t == 6 || t == 2 || t == 4) && m.has_rsec) { sec = (int64_t)m.rsec; nsec = m.rnsec; }
        else if ((t == 5 || t == 1 || t == 3) && m.has_qsec) { sec = (int64_t)m.qsec; nsec = m.qnsec; }
        if (sec < 0) {
            if (!now.tv_sec) timespec_get(&now, TIME_UTC);
            sec = now.tv_sec;
            nsec = now.tv_nsec;
        }
        ssec[j] = sec;
        snsec[j] = nsec;
        e.sec = (uint32_t)sec;
        e.nsec = (uint32_t)nsec;
        e.size = m.frame_len;
        // Net direction by message type (net/v1 :578-597)
        switch (t) {
        case 5: case 10: case 4: case 1: case 8: case 13: case 12: e.dir = 0; break;
        case 9: case 6: case 3: case 2: case 7: case 14: case 11: e.dir = 1; break;
        default: e.dir = 2;
        }
        e.side = (t >= 1 && t <= 14 && (t & 1) == 0) ? 1 : 0; // responses have even type numbers
        e.l3 = m.has_family ? (m.family == 2 ? 6 : (m.family == 1 ? 4 : 0)) : 0;
        e.l4 = m.has_protocol ? (m.protocol == 1 ? 17 : (m.protocol == 2 ? 6 : 0)) : 0;
        e.qport = m.has_qport ? (uint16_t)m.qport : 0;
        e.filtered = (msg_type_mask && !(t < 32 && ((msg_type_mask >> t) & 1))) ? 1 : 0; // a type past the mask's bits never matches
        // deep sampling: each manager draws per dnstap event in stream order (new_event:
        // net/v1 ...cpp:840, dns/v1 ...cpp:1409); a dnstap_msg_type-filtered event is the DNS
        // manager's process_filtered, new_event(stamp, false): no draw, the last flag.
        // pad[0]: bit 0 not deep for the Net manager, bit 1 for the DNS manager
        if (c->sample_rate < 100) {
            const bool net_deep = c->draws_net.next(c->sample_rate);
            if (!e.filtered) c->dns_deep_now = c->draws_dns.next(c->sample_rate);
            e.pad[0] = (uint8_t)((net_deep ? 0u : 1u) | (c->dns_deep_now ? 0u : 2u));
        }
        const uint8_t *msg = nullptr;
        size_t mlen = 0;
        if (c->dns2_groups) {
            // DNS v2 (dns/v2 ...cpp:1176-1270): the transaction direction by message type, a
            // response with its message ends a transaction, else a query message starts one.
            // pad[1]: direction | response << 2 | a message << 3 | socket protocol << 4
            const uint32_t xd = (t == 5 || t == 6 || t == 1 || t == 2 || t == 13 || t == 14) ? 0u
                              : ((t >= 3 && t <= 4) || (t >= 7 && t <= 12)) ? 1u : 2u;
            uint32_t v2 = xd;
            if (e.side == 1 && m.has_rmsg) { v2 |= 4u | 8u; msg = m.rmsg; mlen = m.rmsg_len; }
            else if (m.has_qmsg) { v2 |= 8u; msg = m.qmsg; mlen = m.qmsg_len; }
            if (m.has_protocol && m.protocol >= 1 && m.protocol <= 7) v2 |= (uint32_t)m.protocol << 4;
            e.pad[1] = (uint8_t)v2;
            e.dns_mode = msg ? PV_DT_MESSAGE : PV_DT_EVENT_ONLY;
        } else if (!m.has_qmsg && !m.has_rmsg) e.dns_mode = PV_DT_SIDE;
        else if (e.side == 0 && m.has_qmsg) { e.dns_mode = PV_DT_MESSAGE; msg = m.qmsg; mlen = m.qmsg_len; }
        else if (e.side == 1 && m.has_rmsg) { e.dns_mode = PV_DT_MESSAGE; msg = m.rmsg; mlen = m.rmsg_len; }
        else e.dns_mode = PV_DT_EVENT_ONLY;
        if (mlen > 65535 - 48) mlen = 65535 - 48; // a DNS message fits 16 bits (TCP framing)
        e.qlen = m.has_qaddr ? (uint8_t)std::min<size_t>(m.qaddr.size(), 255) : 0;
        e.rlen = m.has_raddr ? (uint8_t)std::min<size_t>(m.raddr.size(), 255) : 0;
        if (e.qlen == 4 || e.qlen == 16) memcpy(e.qaddr, m.qaddr.data(), e.qlen);
        if (e.rlen == 4 || e.rlen == 16) memcpy(e.raddr, m.raddr.data(), e.rlen);
        // the record: pcap header, IPv4 (or IPv6) header, UDP header, message
        const bool v6 = e.l3 == 6;
        const uint32_t iph = v6 ? 40 : 20;
        const uint32_t incl = iph + 8 + (uint32_t)mlen;
        const size_t r = arena.size();
        arena.resize(r + ((16 + incl + 3) & ~3u), 0);
        uint8_t *h = arena.data() + r;
        const uint32_t hw[4] = {(uint32_t)sec, c->cfg.ts_nano ? (uint32_t)nsec : (uint32_t)(nsec / 1000), incl, incl};
        memcpy(h, hw, 16);
        uint8_t *ip = h + 16;
        const uint32_t udp_len = 8 + (uint32_t)mlen;
        if (v6) {
            ip[0] = 0x60;
            ip[4] = (uint8_t)(udp_len >> 8); ip[5] = (uint8_t)udp_len;
            ip[6] = 17; ip[7] = 64;
            if (e.qlen == 16) memcpy(ip + 8, e.qaddr, 16);
            if (e.rlen == 16) memcpy(ip + 24, e.raddr, 16);
        } else {
            const uint32_t tot = 20 + udp_len;
            ip[0] = 0x45;
            if (tot <= 65535) { ip[2] = (uint8_t)(tot >> 8); ip[3] = (uint8_t)tot; }
            ip[8] = 64; ip[9] = 17;
            if (e.qlen == 4) memcpy(ip + 12, e.qaddr, 4);
            if (e.rlen == 4) memcpy(ip + 16, e.raddr, 4);
        }
        uint8_t *u = ip + iph;
        u[0] = (uint8_t)(e.qport >> 8); u[1] = (uint8_t)e.qport;
        u[2] = 0; u[3] = 53;
        u[4] = (uint8_t)(udp_len >> 8); u[5] = (uint8_t)udp_len;
        if (mlen) memcpy(u + 8, msg, mlen);
        offs[j] = (uint32_t)r;
        e.rec = (uint32_t)r;
        e.moff = (uint32_t)(r + 16 + iph + 8);
        e.mlen = (uint32_t)mlen;
        if (arena.size() > 0xfffff000ull) return c->fail(PV_ECAPACITY, "dnstap events exceed 4 GiB of records");
    }
    arena.resize(arena.size() + PV_RECS_PAD, 0);
    hipError_t e;
    uint8_t *d_arena = nullptr;
    uint32_t *d_offs = nullptr;
    PvDtEv *d_ev = nullptr;
    struct Free {
        void *p[3];
        ~Free() { for (void *q : p) if (q) hipFree(q); }
    } fr{{nullptr, nullptr, nullptr}};
    if (!hip_ok(e = hipMalloc(&d_arena, arena.size())) || !hip_ok(e = hipMalloc(&d_offs, n * 4)) ||
        !hip_ok(e = hipMalloc(&d_ev, n * sizeof(PvDtEv))))
        return c->hipfail(e, "dnstap buffers");
    fr.p[0] = d_arena; fr.p[1] = d_offs; fr.p[2] = d_ev;
    hipStream_t st = c->stream;
    if (!hip_ok(e = hipMemcpyAsync(d_arena, arena.data(), arena.size(), hipMemcpyHostToDevice, st)) ||
        !hip_ok(e = hipMemcpyAsync(d_offs, offs.data(), n * 4, hipMemcpyHostToDevice, st)) ||
        !hip_ok(e = hipMemcpyAsync(d_ev, ev.data(), n * sizeof(PvDtEv), hipMemcpyHostToDevice, st)))
        return c->hipfail(e, "dnstap H2D");
    ensure_started(c, ssec[0], snsec[0]);
    const uint32_t np = c->cfg.num_periods;
    auto span = [&](size_t a, size_t b) -> int {
        if (b <= a) return 0;
        PvParams P;
        params_common(c, P, d_arena, d_offs + a, b - a);
        P.linktype = 101;
        P.tap = 1;
        P.f_flags = 0; // the DNS filters do not apply to dnstap events (only dnstap_msg_type)
        P.dq = reinterpret_cast<uint64_t *>(d_ev + a);
        P.gbase = c->global_base + c->records_seen;
        P.slot_of[0] = c->net.slot_at(0);
        P.dslot_of[0] = c->dns.slot_at(0);
        P.sum = c->d_sum;
        P.cpc = c->d_cpc;
        P.tkeys = c->d_tkeys;
        P.tcnt = c->d_tcnt;
        P.taux = c->d_taux;
        P.tcap_log2 = c->tcap_log2;
        P.reg_log2 = c->reg_log2;
        P.arena = c->d_arena;
        P.arena_top = c->d_arena_top;
        P.arena_cap = c->arena_cap;
        P.flags = c->d_status + ST_FLAGS;
        P.tab_live = c->d_tab_live;
        P.ovf = c->d_ovf;
        P.ovf_cnt = c->d_ovf_cnt;
        P.ovf_cap = c->ovf_cap;
        const uint32_t blocks = (uint32_t)((b - a + 255) / 256);
        // DNS v2: transaction events, one 256-event region per block (pv_xact_compact), paired by
        // the transaction stage as a pcap batch's are
        P.want_events = c->dns2_groups ? 1u : 0u;
        if (P.want_events) {
            if (b - a > c->max_records) return c->fail(PV_ECAPACITY, "a dnstap period span exceeds max_records events");
            P.events = c->d_events;
            P.eecs = c->d_eecs;
            P.ekeys = c->d_ekeys;
            P.blk_events = c->d_blk_events;
            P.skeys = c->d_skeys;
            P.svals = c->d_svals;
            P.n_events = c->d_status + ST_NEV;
            P.n_keys = c->d_status + ST_NKEYS;
            P.wt_per_block = 4; // 64-record tiles: 256 events per block
            P.grid_main = blocks;
            if (c->n_pend == 0) c->pend_base = (int64_t)c->records_seen - 1;
            P.ekey_base = (uint32_t)((int64_t)c->records_seen - c->pend_base);
            launch_fill32(c, c->d_status, ST_ALLOC, 0);
        }
        launch_fill32(c, c->d_status + ST_FLAGS, 1, 0);
        flush_fills(c);
        *c->h_params = P;
        if (!hip_ok(e = upload_params(c->d_params, c->h_params, sizeof P, st)))
            return c->hipfail(e, "parameter upload");
        hipLaunchKernelGGL(pv_dnstap_kernel, dim3(blocks), dim3(256), 0, st, (const PvParams *)c->d_params);
        if (P.want_events) hipLaunchKernelGGL(pv_xact_compact, dim3(blocks), dim3(256), 0, st, (const PvParams *)c->d_params, 0u, 0u);
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "pv_dnstap_kernel");
        if (P.want_events) {
            const uint32_t nev = c->h_status[ST_NEV], nresp = c->h_status[ST_NRESP];
            if (int rc = pair_stage(c, P, nev, c->h_status[ST_NKEYS], nresp, b - a, st, (uint64_t)blocks * P.wt_per_block * 64u))
                return rc;
        }
        if (int rc = drain_overflow(c, st)) return rc;
        uint32_t flags = 0;
        if (!hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
        if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
        if (flags & PVF_ARENA_FULL) return c->fail(PV_ECAPACITY, "top-N name arena full");
        c->net.clean[P.slot_of[0]] = false;
        c->dns.clean[P.dslot_of[0]] = false;
        c->records_seen += b - a;
        return purge_tables(c, st);
    };
    size_t a = 0;
    for (size_t j = 0; j < n; j++) {
        // each manager shifts on the first of its events at or after its next shift
        // (AbstractMetricsManager::new_event, src/AbstractMetricsManager.h:318-333)
        const bool ns = np > 1 && ssec[j] >= c->net.next_shift_sec;
        const bool ds = np > 1 && ssec[j] >= c->dns.next_shift_sec;
        if (!ns && !ds) continue;
        if (int rc = span(a, j)) return rc;
        if (ns) { clear_part(c, PART_NET, c->net.slot_at(1)); win_shift(c, c->net, ssec[j]); }
        if (ds && c->dns2_groups) {
            // DNS v2's on_period_shift purge of the open transactions (as a heartbeat shift)
            if (int rc = dns_period_shift(c, ssec[j], snsec[j])) return rc;
        } else if (ds) { clear_part(c, PART_DNS, c->dns.slot_at(1)); win_shift(c, c->dns, ssec[j]); }
        a = j;
    }
    if (int rc = span(a, n)) return rc;
    c->last_sec = ssec[n - 1];
    c->last_nsec = snsec[n - 1];
    return 0;
}

// pcapng -> classic pcap records with nanosecond fractions (pv_pcapng.cpp). out == NULL (or too
// small): only *out_bytes / *n_records are set (PV_ECAPACITY when out is too small).
int pv_pcapng_records(const uint8_t *buf, size_t bytes, uint8_t *out, size_t out_cap, size_t *out_bytes,
                      uint32_t *linktype, uint64_t *n_records)
{
    std::vector<uint8_t> v;
    const int rc = pvi::pcapng_to_records(buf, bytes, &v, linktype, n_records);
    if (rc == pvi::PVNG_ELINKTYPES) return PV_EUNSUPPORTED;
    if (rc) return PV_EINVAL;
    *out_bytes = v.size();
    if (!out) return 0;
    if (out_cap < v.size()) return PV_ECAPACITY;
    memcpy(out, v.data(), v.size());
    return 0;
}

// One TPACKET_V3 ring block (AFPacket::walk_block, src/inputs/pcap/afpacket.cpp:72-86) ->
// classic pcap records with nanosecond fractions, appended at out + *out_bytes. As the
// reference hands them on, every packet takes the block's ts_last_pkt (not its own tp_sec /
// tp_nsec) and its snap length as both lengths (RawPacket(data, tp_snaplen, ...)).
int pv_tpacket3_block_records(const uint8_t *block, size_t block_size, uint8_t *out, size_t out_cap, size_t *out_bytes,
                              uint64_t *n_records)
{
    if (block_size < sizeof(tpacket_block_desc)) return PV_EINVAL;
    const tpacket_block_desc *bd = reinterpret_cast<const tpacket_block_desc *>(block);
    const tpacket_hdr_v1 &h = bd->hdr.bh1;
    const uint32_t ts_sec = h.ts_last_pkt.ts_sec, ts_nsec = h.ts_last_pkt.ts_nsec;
    size_t o = *out_bytes;
    uint64_t n = 0;
    size_t p = h.offset_to_first_pkt;
    for (uint32_t i = 0; i < h.num_pkts; i++) {
        if (p + sizeof(tpacket3_hdr) > block_size) return PV_EINVAL;
        tpacket3_hdr ph;
        memcpy(&ph, block + p, sizeof ph);
        const size_t d = p + ph.tp_mac;
        if (d + ph.tp_snaplen > block_size) return PV_EINVAL;
        if (o + 16 + ph.tp_snaplen > out_cap) return PV_ECAPACITY;
        const uint32_t rh[4] = {ts_sec, ts_nsec, ph.tp_snaplen, ph.tp_snaplen};
        memcpy(out + o, rh, 16);
        memcpy(out + o + 16, block + d, ph.tp_snaplen);
        o += 16 + ph.tp_snaplen;
        n++;
        if (i + 1 < h.num_pkts && ph.tp_next_offset == 0) return PV_EINVAL;
        p += ph.tp_next_offset;
    }
    *out_bytes = o;
    if (n_records) *n_records += n;
    return 0;
}

// Frame Streams decode only (tests): data frames read and dnstap MESSAGE events found.
int pv_dnstap_count(const uint8_t *buf, size_t bytes, uint32_t *frames, uint32_t *events)
{
    std::vector<pvi::DtMessage> msgs;
    pvi::dnstap_decode(buf, bytes, msgs, frames);
    *events = (uint32_t)msgs.size();
    return 0;
}

// Host-memory path with the record index on the device. The blob is cut into fixed
// chunk-sized pieces in host order, so their H2D copies stream back to back (a producer
// thread, two copy streams, a ring of ring_n device buffers of two chunks each) without
// waiting on any index. The calling thread, per piece: moves the previous batch's tail (the
// records after its last ts_sec cut) in front of the piece on the device, indexes the joined
// run there (pv_index.hip), cuts it at its last ts_sec boundary and runs the batch. The host
// reads a few header words only. Batches are cut as pv_process_host's host-index path cuts
// them (at most stage_recs records, ending at a ts_sec boundary unless the data ends).
int process_host_ring(pv_ctx *c, const uint8_t *recs, size_t bytes)
{
    const size_t L = c->stage_bytes; // a multiple of 256: runs start 256-B aligned (+ first)
    hipError_t e;
    const uint32_t NR = c->ring_n;
    for (uint32_t q = 0; q < NR; q++) {
        pv_ctx::Ring &r = c->ring[q];
        if (r.d_buf) continue;
        if (!hip_ok(e = hipMalloc(&r.d_buf, 2 * L + PV_RECS_PAD)) || !hip_ok(e = hipMalloc(&r.d_offs, c->stage_recs * 4)) ||
            !hip_ok(e = hipEventCreateWithFlags(&r.landed, hipEventDisableTiming)) ||
            // on the context's stream: a null-stream memset is not ordered with the
            // non-blocking copy streams and could land after a piece's copy
            !hip_ok(e = hipMemsetAsync(r.d_buf, 0, 2 * L + PV_RECS_PAD, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "ingest ring");
    }
    if (!c->copy_stream2 && !hip_ok(e = hipStreamCreateWithFlags(&c->copy_stream2, hipStreamNonBlocking)))
        return c->hipfail(e, "copy stream");
    const bool pinned = host_pinned(recs);
    if (!pinned)
        for (uint32_t q = 0; q < NR; q++)
            if (!c->ring[q].h_stage && !hip_ok(e = hipHostMalloc((void **)&c->ring[q].h_stage, L, hipHostMallocDefault)))
                return c->hipfail(e, "ingest staging");
    const uint64_t npieces = (bytes + L - 1) / L;
    // producer: piece p's copy into ring slot p % NR at offset L. Slot p % NR last held run
    // p - NR, whose batches are done and whose tail run p - NR + 1 has moved out: issued once the
    // consumer has finished run p - NR + 1 (freed > p - NR), so up to NR - 2 pieces ahead of it. The consumer synchronises its stream
    // after each run, so the host-side order is the device-side order.
    std::mutex mu;
    std::condition_variable cv;
    uint64_t issued = 0, freed = 0;
    bool abort = false;
    int prod_rc = 0;
    std::string prod_err;
    auto producer = [&] {
        for (uint64_t k = 0; k < npieces; k++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return abort || k < freed + NR; });
                if (abort) return;
            }
            pv_ctx::Ring &r = c->ring[k % NR];
            const size_t len = std::min(L, bytes - k * L);
            const uint8_t *src = recs + k * L;
            if (!pinned) {
                auto t1 = std::chrono::steady_clock::now();
                pvi::copy_parallel(*c->pool, r.h_stage, src, len);
                src = r.h_stage;
                c->ingest_ms[0] += ms_since(t1);
            }
            hipStream_t cs = (k & 1) ? c->copy_stream2 : c->copy_stream;
            const auto ti = std::chrono::steady_clock::now();
            const bool ok = hip_ok(e = hipMemcpyAsync(r.d_buf + L, src, len, hipMemcpyHostToDevice, cs)) &&
                            hip_ok(e = hipEventRecord(r.landed, cs));
            c->ingest_ms[2] += ms_since(ti); // host time the copy's issue takes (a blocking copy shows here)
            if (!ok) {
                std::lock_guard<std::mutex> g(mu);
                prod_rc = PV_EHIP;
                prod_err = std::string("H2D: ") + hipGetErrorString(e);
                abort = true;
                cv.notify_all();
                return;
            }
            std::lock_guard<std::mutex> g(mu);
            issued = k + 1;
            cv.notify_all();
        }
    };
    std::thread th(producer);
    pv_ctx::Stage &st = c->stage[0]; // index state, change lists, host offsets (fallback)
    int rc = 0;
    size_t tail = 0;
    const uint8_t *tail_src = nullptr;
    for (uint64_t k = 0; k < npieces && !rc; k++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return abort || issued > k; });
            if (abort) break;
        }
        HP(0);
        pv_ctx::Ring &r = c->ring[k % NR];
        const size_t len = std::min(L, bytes - k * L);
        const bool last_piece = k + 1 == npieces;
        // the run: the tail at [L - tail, L), the piece at [L, L + len); b is 256-B aligned and
        // the first record at b + first; hf is that record in host memory
        uint8_t *b = r.d_buf + ((L - tail) & ~(size_t)255);
        uint32_t first = (uint32_t)((L - tail) & 255);
        const uint8_t *hf = recs + k * L - tail;
        size_t end = first + tail + len;
        auto t0 = std::chrono::steady_clock::now();
        if (!hip_ok(e = hipStreamWaitEvent(c->stream, r.landed, 0)) ||
            (tail && !hip_ok(e = hipMemcpyAsync(b + first, tail_src, tail, hipMemcpyDeviceToDevice, c->stream)))) {
            rc = c->hipfail(e, "ingest run");
            break;
        }
        tail = 0;
        for (;;) {
            bool capped = false;
            int ix = device_index(c, st, b, first, hf, end, r.d_offs, c->stream, &capped);
            if (ix < 0) { rc = ix; break; }
            if (ix > 0 && (rc = host_index_run(c, st, b, first, hf, end, r.d_offs, &capped))) break;
            pv_index_info info = st.info;
            c->ingest_ms[1] += ms_since(t0);
            HP(1);
            const bool more = !last_piece || capped; // records follow this batch
            if (info.n_records == 0) {
                if (!last_piece && end - first >= L) { rc = c->fail(PV_ECAPACITY, "record larger than the ingest chunk"); break; }
                if (!last_piece) { tail = end - first; tail_src = b + first; }
                break;
            }
            // a batch that more records follow ends at its last ts_sec boundary when it spans
            // more than one second, so a period shift and the DNS records of its first second
            // reach the device in the same batch
            if (more && info.n_sec_changes > 1 && info.n_sec_changes <= st.sci.size()) {
                const uint32_t cut = st.sci[info.n_sec_changes - 1];
                const uint32_t o[2] = {st.cut_o[0], st.cut_o[1]}; // the offsets either side of the cut
                info.n_records = cut;
                info.bytes_used = o[1];
                info.n_sec_changes -= 1;
                uint32_t h[2];
                memcpy(h, hf + (o[0] - first), 8);
                info.last_sec = h[0];
                info.last_nsec = c->cfg.ts_nano ? (int64_t)h[1] : (int64_t)h[1] * 1000;
                capped = true;
            }
            auto t2 = std::chrono::steady_clock::now();
            HP(2);
            c->eoc_batch = c->eoc_armed && !capped && last_piece; // the data ends with this batch
            rc = pv_process_device(c, b, r.d_offs, &info, st.sci.data(), st.scs.data(), nullptr);
            if (!rc) rc = pv_synchronize(c);
            HP(8);
            c->ingest_ms[3] += ms_since(t2);
            if (rc) break;
            t0 = std::chrono::steady_clock::now();
            const size_t used = info.bytes_used;
            const size_t rest = end - used;
            if (!capped && last_piece) break;          // the data ends (at most a partial record)
            if (!last_piece && (!capped || rest <= L)) {
                if (rest > L) { rc = c->fail(PV_ECAPACITY, "record larger than the ingest chunk"); break; }
                tail = rest;
                tail_src = b + used;
                break;
            }
            // more batches from this run, in place
            hf += used - first;
            b += used & ~(size_t)255;
            first = (uint32_t)(used & 255);
            end -= used & ~(size_t)255;
        }
        {
            std::lock_guard<std::mutex> g(mu);
            freed = k; // slot (k - 1) % NR is free: its tail has moved into this run
            cv.notify_all();
        }
        HP(9);
    }
    {
        std::lock_guard<std::mutex> g(mu);
        if (rc) abort = true;
        freed = npieces + NR;
        cv.notify_all();
    }
    th.join();
    hipStreamSynchronize(c->copy_stream);
    hipStreamSynchronize(c->copy_stream2);
    if (rc) return rc;
    if (prod_rc) return c->fail(prod_rc, "%s", prod_err.c_str());
    return 0;
}

// Host-memory path, pipelined over chunks of the record blob: a producer thread stages
// chunk k + 1 (parallel copy into pinned memory unless the caller's buffer is already
// pinned, parallel record index, H2D on the copy stream) while the calling thread runs
// chunk k's kernels. Results equal one pv_process_device per chunk, in order.
int pv_set_bpf(pv_ctx *c, const pv_bpf_insn *prog, uint32_t n)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (n == 0) { c->bpf.clear(); return 0; }
    if (pv_bpf_validate(prog, n)) return c->fail(PV_EINVAL, "invalid BPF program (classic-BPF checker)");
    c->bpf.assign(prog, prog + n);
    c->bpf_dirty = true;
    return 0;
}

namespace {
int process_host_block(pv_ctx *c, const uint8_t *recs, size_t bytes);
}

int pv_process_host(pv_ctx *c, const uint8_t *recs, size_t bytes)
{
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (int rc = merged_refuse(c)) return rc;
        c->in_host = true;
    }
    // (the pcap input's BPF filter, PcapInputStream.cpp:485-488, runs on the device on each batch:
    // pv_process_device)
    const int rc = process_host_block(c, recs, bytes);
    std::lock_guard<std::mutex> g(c->mu);
    c->in_host = false;
    c->eoc_armed = c->eoc_batch = c->eoc_stage = false;
    return rc;
}

namespace {
int process_host_block(pv_ctx *c, const uint8_t *recs, size_t bytes)
{
    hipSetDevice(c->device);
    if (int rc = ingest_setup(c)) return rc;
    if (c->device_index && bytes >= 4096) return process_host_ring(c, recs, bytes);
    const bool pinned = host_pinned(recs);
    std::mutex mu;
    std::condition_variable cv;
    int state[2] = {0, 0};        // 0 free, 1 ready
    bool prod_done = false, abort = false;
    uint64_t nchunks = 0;
    int prod_rc = 0;
    std::string prod_err;
    auto producer = [&] {
        size_t pos = 0;
        uint64_t k = 0;
        int rc = 0;
        while (pos < bytes) {
            pv_ctx::Stage &st = c->stage[k & 1];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return state[k & 1] == 0 || abort; });
                if (abort) break;
            }
            const size_t L = std::min(c->stage_bytes, bytes - pos);
            const uint8_t *src = recs + pos;
            auto t1 = std::chrono::steady_clock::now();
            // pageable source: copied into pinned staging by the threads that index it
            rc = pvi::index_records_parallel(*c->pool, src, L, c->cfg.ts_nano, st.h_offs, c->stage_recs, st.sci.data(),
                                             st.scs.data(), (uint32_t)st.sci.size(), &st.info, pinned ? nullptr : st.h_recs);
            if (rc) { prod_err = "record index failed"; break; }
            const uint8_t *base = pinned ? src : st.h_recs;
            c->ingest_ms[pinned ? 1 : 0] += ms_since(t1);
            if (st.info.n_records == 0) {
                if (L == c->stage_bytes && pos + L < bytes) { rc = PV_ECAPACITY; prod_err = "record larger than the ingest chunk"; }
                break;
            }
            // a chunk that is not the last ends at a ts_sec boundary when it spans more than
            // one second, so a period shift and the DNS records of its first second reach
            // the device in the same batch
            if (pos + st.info.bytes_used < bytes && st.info.n_sec_changes > 1 &&
                st.info.n_sec_changes <= st.sci.size()) {
                const uint32_t last = st.sci[st.info.n_sec_changes - 1];
                st.info.n_records = last;
                st.info.bytes_used = st.h_offs[last];
                st.info.n_sec_changes -= 1;
                const uint32_t prev = st.h_offs[last - 1];
                uint32_t h[2];
                memcpy(h, base + prev, 8);
                st.info.last_sec = h[0];
                st.info.last_nsec = c->cfg.ts_nano ? (int64_t)h[1] : (int64_t)h[1] * 1000;
            }
            auto t2 = std::chrono::steady_clock::now();
            const size_t used = st.info.bytes_used;
            hipError_t e = hipSuccess;
            const bool ok = hip_ok(e = hipMemcpyAsync(st.d_recs, base, used, hipMemcpyHostToDevice, c->copy_stream)) &&
                             hip_ok(e = hipMemsetAsync(st.d_recs + used, 0, PV_RECS_PAD, c->copy_stream)) &&
                             hip_ok(e = hipMemcpyAsync(st.d_offs, st.h_offs, st.info.n_records * 4, hipMemcpyHostToDevice,
                                                       c->copy_stream));
            if (!ok || !hip_ok(e = hipEventRecord(st.copied, c->copy_stream))) {
                rc = PV_EHIP;
                prod_err = std::string("H2D: ") + hipGetErrorString(e);
                break;
            }
            c->ingest_ms[2] += ms_since(t2);
            pos += used;
            // the final batch: no complete record follows (at most a partial one)
            {
                const size_t rest = bytes - pos;
                uint32_t cl = 0;
                if (rest >= 16) memcpy(&cl, recs + pos + 8, 4);
                st.last = rest < 16 || 16 + (size_t)cl > rest;
            }
            std::lock_guard<std::mutex> g(mu);
            state[k & 1] = 1;
            k++;
            cv.notify_all();
        }
        std::lock_guard<std::mutex> g(mu);
        prod_rc = rc;
        prod_done = true;
        nchunks = k;
        cv.notify_all();
    };
    std::thread th(producer);
    int rc = 0;
    for (uint64_t k = 0;; k++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return state[k & 1] == 1 || (prod_done && k >= nchunks); });
            if (state[k & 1] != 1) break;
        }
        pv_ctx::Stage &st = c->stage[k & 1];
        auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipStreamWaitEvent(c->stream, st.copied, 0);
        if (!hip_ok(e)) rc = c->hipfail(e, "stream wait");
        c->eoc_batch = c->eoc_armed && st.last;
        if (!rc) rc = pv_process_device(c, st.d_recs, st.d_offs, &st.info, st.sci.data(), st.scs.data(), nullptr);
        if (!rc) rc = pv_synchronize(c);
        c->ingest_ms[3] += ms_since(t0);
        std::lock_guard<std::mutex> g(mu);
        state[k & 1] = 0;
        if (rc) abort = true;
        cv.notify_all();
        if (rc) break;
    }
    th.join();
    hipStreamSynchronize(c->copy_stream);
    if (rc) return rc;
    if (prod_rc) return c->fail(prod_rc, "%s", prod_err.c_str());
    return 0;
}
} // namespace

// The device record index (pv_index.hip) of one block in host memory, filled as
// pv_index_records fills its outputs (a block of at most one ingest chunk).
int pv_index_records_device(pv_ctx *c, const uint8_t *recs, size_t bytes, uint32_t *offsets, uint64_t max_records,
                            uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes, pv_index_info *info)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = ingest_setup(c)) return rc;
    if (bytes > c->stage_bytes) return c->fail(PV_EINVAL, "block of %zu bytes exceeds the ingest chunk", bytes);
    if (bytes < 16) { // no complete record header
        memset(info, 0, sizeof *info);
        info->monotone = 1;
        return 0;
    }
    pv_ctx::Stage &st = c->stage[0];
    hipError_t e;
    if (!hip_ok(e = hipMemcpyAsync(st.d_recs, recs, bytes, hipMemcpyHostToDevice, c->copy_stream)) ||
        !hip_ok(e = hipMemsetAsync(st.d_recs + bytes, 0, PV_RECS_PAD, c->copy_stream)))
        return c->hipfail(e, "H2D");
    bool capped = false;
    hipStreamSynchronize(c->copy_stream);
    int rc = device_index(c, st, st.d_recs, 0, recs, bytes, st.d_offs, c->stream, &capped);
    if (rc < 0) return rc;
    if (rc > 0 && (rc = host_index_run(c, st, st.d_recs, 0, recs, bytes, st.d_offs, &capped))) return rc;
    const uint64_t n = std::min<uint64_t>(st.info.n_records, max_records);
    if (n && (!hip_ok(e = hipMemcpyAsync(offsets, st.d_offs, n * 4, hipMemcpyDeviceToHost, c->copy_stream)) ||
              !hip_ok(e = hipStreamSynchronize(c->copy_stream))))
        return c->hipfail(e, "D2H offsets");
    *info = st.info;
    info->n_records = n;
    uint32_t nch = (uint32_t)st.info.n_sec_changes;
    if (n && n < st.info.n_records) {
        // capped at max_records: the walk as pv_index_records stops it there
        uint32_t hl[4];
        memcpy(hl, recs + offsets[n - 1], 16);
        info->bytes_used = offsets[n - 1] + 16 + (uint64_t)hl[2];
        info->last_sec = hl[0];
        info->last_nsec = c->cfg.ts_nano ? (int64_t)hl[1] : (int64_t)hl[1] * 1000;
        while (nch && st.sci[nch - 1] >= n) nch--;
        info->n_sec_changes = nch;
        // monotonicity of the first n records
        info->monotone = 1;
        for (uint32_t k = 1; k < nch; k++)
            if (st.scs[k] < st.scs[k - 1]) info->monotone = 0;
    }
    const uint32_t nc = std::min<uint32_t>(nch, max_changes);
    for (uint32_t k = 0; k < nc; k++) { sc_idx[k] = st.sci[k]; sc_sec[k] = st.scs[k]; }
    return nch > max_changes ? PV_ECAPACITY : 0;
}

int pv_ingest_timing(pv_ctx *c, double *ms4, int reset)
{
    for (int i = 0; i < 4; i++) ms4[i] = c->ingest_ms[i];
    if (reset) for (double &v : c->ingest_ms) v = 0;
    return 0;
}

int pv_host_register(void *p, size_t bytes)
{
    return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? 0 : PV_EHIP;
}

int pv_host_unregister(void *p)
{
    return hipHostUnregister(p) == hipSuccess ? 0 : PV_EHIP;
}

int pv_index_records_mt(const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets, uint64_t max_records,
                        uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes, pv_index_info *info,
                        uint32_t nthreads)
{
    pvi::Pool pool(nthreads ? nthreads : pvi::default_threads());
    return pvi::index_records_parallel(pool, recs, bytes, ts_nano, offsets, max_records, sc_idx, sc_sec, max_changes,
                                       info);
}

int pv_set_start_tstamp(pv_ctx *c, int64_t sec, int64_t nsec)
{
    std::lock_guard<std::mutex> g(c->mu);
    return ensure_started(c, sec, nsec);
}

int pv_set_end_tstamp(pv_ctx *c, int64_t sec, int64_t nsec)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->started) return 0;
    // end_tstamp_signal: the live bucket of each manager becomes read-only
    c->net.meta[c->net.slots.front()].set_read_only(sec, nsec);
    c->dns.meta[c->dns.slots.front()].set_read_only(sec, nsec);
    c->ended = true;
    return 0;
}

// heartbeat_signal -> StreamMetricsHandler::check_period_shift in both handlers
// (src/AbstractMetricsManager.h:462-470; net/v1/NetStreamHandler.cpp:99-102,
// dns/v1/DnsStreamHandler.cpp:219-222): each manager shifts its window at `stamp` when
// num_periods > 1 and stamp.sec has reached its next shift, with no event. The DNS manager's
// on_period_shift (dns/v1/DnsStreamHandler.h:252-267; v2 .h:440-453) then purges the open
// transactions the stamp expires (timed out in the new live bucket) and takes the slow
// thresholds from the bucket just closed.
int pv_check_period_shift(pv_ctx *c, int64_t sec, int64_t nsec)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = merged_refuse(c)) return rc;
    hipSetDevice(c->device);
    if (!c->started || c->cfg.num_periods <= 1) return 0;
    if (sec >= c->net.next_shift_sec) {
        clear_part(c, PART_NET, c->net.slot_at(1));
        c->net.clean[c->net.slot_at(1)] = false;
        win_shift(c, c->net, sec, nsec);
    }
    if (sec < c->dns.next_shift_sec) return 0;
    return dns_period_shift(c, sec, nsec);
}

// The DNS manager's shift at `sec` with no event (a heartbeat, or a dnstap span boundary): the
// new live bucket, DnsMetricsManager::on_period_shift's purge of the open transactions through
// the pairing stage, the slow thresholds of the bucket just closed
int dns_period_shift(pv_ctx *c, int64_t sec, int64_t nsec)
{
    hipStream_t st = c->stream;
    const uint32_t s0 = c->dns.slot_at(0), s1 = c->dns.slot_at(1);
    clear_part(c, PART_DNS, s1);
    c->dns.clean[s1] = false;
    const bool xacts = (c->dns_groups & PV_DNS_TRANSACTIONS) || c->dns2_groups;
    if (xacts && c->n_pend > 0) {
        // the carried queries through the pairing stage with one shift at the stamp and no
        // events: purge_period() times out those with stamp.sec >= ttl_s + start.sec
        PvParams P;
        params_common(c, P, nullptr, nullptr, 0);
        P.n_dshift = 1;
        P.dthresh[0] = sec;
        P.dskip_before = 0;
        P.dslot_of[0] = s0;
        P.dslot_of[1] = s1;
        P.slot_of[0] = c->net.slot_at(0);
        P.sum = c->d_sum;
        P.cpc = c->d_cpc;
        P.tkeys = c->d_tkeys;
        P.tcnt = c->d_tcnt;
        P.taux = c->d_taux;
        P.tcap_log2 = c->tcap_log2;
        P.reg_log2 = c->reg_log2;
        P.arena = c->d_arena;
        P.arena_top = c->d_arena_top;
        P.arena_cap = c->arena_cap;
        P.tab_live = c->d_tab_live; // global_add counts the entries it creates
        P.events = c->d_events;
        P.eecs = c->d_eecs;
        P.gbase = c->global_base + c->records_seen;
        P.ekey_base = (uint32_t)((int64_t)c->records_seen - c->pend_base);
        P.flags = c->d_status + ST_FLAGS;
        flush_fills(c);
        if (int rc = pair_stage(c, P, 0, 0, 0, 0, st, 0)) return rc;
    } else if (xacts && ((c->dns_groups & PV_DNS_QUANTILES) || (c->dns2_groups & PV_DNS2_XACT_TIMES))) {
        // nothing open: only the slow thresholds of the closed bucket (kept when it had none)
        if (int rc = sync_xvals(c)) return rc;
        const uint32_t sg = s0 | (c->gen[s0] << 8);
        std::vector<uint64_t> fr, to, t2[3];
        for (auto &v : c->xvals_host) {
            if (v.slot != sg) continue;
            if (v.kind == XV_FROM_US) fr.push_back(v.bits);
            else if (v.kind == XV_TO_US) to.push_back(v.bits);
            else if (v.kind >= XV2_TIME && v.kind < XV2_TIME + 3) t2[v.kind - XV2_TIME].push_back(v.bits);
        }
        if (!fr.empty()) c->from90 = (float)quantile_at(fr, 0.90);
        if (!to.empty()) c->to90 = (float)quantile_at(to, 0.90);
        for (uint32_t d = 0; d < 3; d++)
            if (!t2[d].empty()) c->p90_2[d] = (float)quantile_at(t2[d], 0.90);
    }
    win_shift(c, c->dns, sec, nsec);
    c->dns_shifts.emplace_back(sec, c->dns.slot_at(0));
    c->dns_shift_ord.emplace_back(sec, c->dns.ordinal);
    flush_fills(c);
    hipError_t e = hipStreamSynchronize(st);
    return hip_ok(e) ? 0 : c->hipfail(e, "heartbeat period shift");
}

int pv_window_json(pv_ctx *c, uint32_t period, int merged, char **out)
{
    *out = nullptr;
    // the transaction values are drained under the lock: a batch the producer runs between
    // the drain and the read would otherwise show its counters without its values
    std::lock_guard<std::mutex> g(c->mu);
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    Json j;
    j.obj();
    std::vector<uint32_t> slots;
    {
        if ((rc = window_slots(c, c->net, period, merged != 0, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, merged != 0, PART_NET, b))) return rc;
        j.key("packets").obj();
        net_json(c, j, b);
        j.end_obj();
        if (c->net2_groups) {
            j.key("net").obj();
            net2_json(c, j, b);
            j.end_obj();
        }
    }
    {
        if ((rc = window_slots(c, c->dns, period, merged != 0, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, merged != 0, PART_DNS, b))) return rc;
        j.key("dns").obj();
        if (c->dns2_groups) dns2_json(c, j, b);
        else dns_json(c, j, b);
        j.end_obj();
    }
    j.end_obj();
    *out = strdup(j.s.c_str());
    return 0;
}

// ---- external buckets: the bucket half of the handler object (StreamHandler::merge and the
// window_*(..., AbstractMetricsBucket *) overloads, src/StreamHandler.h:72-77,221-269), which
// a policy uses to fold like handlers across taps (Policy::_get_merged_buckets,
// src/Policies.cpp:420-446)
} // extern "C"
struct pv_bucket {
    int part;            // PART_NET / PART_DNS
    uint32_t handler;    // PV_HANDLER_NET / PV_HANDLER_DNS
    HostBucket b;
};
namespace {
// Quantile::merge(other, Aggregate::SUM) (src/Metrics.h:356-372) on exact values: the sketch of
// a non-empty bucket stays, the p-wise sum of the quantiles grows; an empty one merges
template <typename T>
void qsum_fold(std::vector<T> &dv, std::vector<T> &qs, const std::vector<T> &ov, const std::vector<T> &oqs)
{
    if (dv.empty()) { dv.insert(dv.end(), ov.begin(), ov.end()); return; }
    if (ov.empty()) return;
    const std::vector<T> oq = quantiles(ov);
    (void)oqs; // the other sketch's own quantiles (get_quantiles(other._quantile)), not its sums
    if (qs.empty()) qs = quantiles(dv);
    for (int i = 0; i < 4; i++) qs[i] += oq[i];
}
// AbstractMetricsBucket::merge(other, Aggregate::SUM) (src/AbstractMetricsManager.h:177-195) and
// the handlers' specialized_merge (net/v1/NetStreamHandler.cpp:285-330,
// dns/v1/DnsStreamHandler.cpp:658-733)
void bucket_fold_sum(HostBucket &d, const HostBucket &o, int part)
{
    d.period_length += o.period_length;
    if (o.start_sec < d.start_sec) { d.start_sec = o.start_sec; d.start_nsec = o.start_nsec; }
    if (o.end_sec > d.end_sec) { d.end_sec = o.end_sec; d.end_nsec = o.end_nsec; }
    // payload_size, a Quantile over a dense histogram: an empty one merges the other's sketch,
    // else the p-wise sums grow
    auto payload_fold = [&](size_t off, std::vector<uint64_t> &qs) {
        uint64_t dn = 0, on = 0;
        const auto dq = hist_quantiles(&d.sum[off], PV_PAYLOAD_BINS, dn);
        const auto oq = hist_quantiles(&o.sum[off], PV_PAYLOAD_BINS, on);
        if (!dn) {
            for (size_t i = 0; i < PV_PAYLOAD_BINS; i++) d.sum[off + i] += o.sum[off + i];
        } else if (on) {
            if (qs.empty()) qs = dq;
            for (int i = 0; i < 4; i++) qs[i] += oq[i];
        }
    };
    if (part == PART_NET) {
        // counters (v1, and v2's per direction); Net v2 specialized_merge
        // (net/v2/NetStreamHandler.cpp:286-331): per direction the same rules
        for (size_t i = 0; i < PV_SUM_NET_WORDS; i++)
            if ((i < PV_OFF_PAYLOAD || i >= PV_OFF_PAYLOAD + PV_PAYLOAD_BINS) && i < PV_OFF_PAYLOAD2) d.sum[i] += o.sum[i];
        payload_fold(PV_OFF_PAYLOAD, d.qs_payload);
        for (uint32_t x = 0; x < 3; x++) payload_fold(PV_OFF_PAYLOAD2 + x * PV_PAYLOAD_BINS, d.qs_payload2[x]);
    } else {
        for (size_t i = PV_OFF_DNS; i < PV_SUM_WORDS; i++) d.sum[i] += o.sum[i];
        // histograms merge their sketches; the quantiles follow the SUM rule
        if (!d.hist_sep) { d.hfrom_us = d.from_us; d.hto_us = d.to_us; d.hist_sep = true; }
        const auto &ohf = o.hist_from(), &oht = o.hist_to();
        d.hfrom_us.insert(d.hfrom_us.end(), ohf.begin(), ohf.end());
        d.hto_us.insert(d.hto_us.end(), oht.begin(), oht.end());
        qsum_fold(d.from_us, d.qs_from, o.from_us, o.qs_from);
        qsum_fold(d.to_us, d.qs_to, o.to_us, o.qs_to);
        qsum_fold(d.ratio, d.qs_ratio, o.ratio, o.qs_ratio);
        // DNS v2 specialized_merge (dns/v2/DnsStreamHandler.cpp:619-676), per direction:
        // dnsTimeUs and dnsRatio by the SUM rule, dnsHistTimeUs merging its sketch
        if (!d.hist2_sep) {
            for (uint32_t x = 0; x < 3; x++) d.htime2[x] = d.time2[x];
            d.hist2_sep = true;
        }
        for (uint32_t x = 0; x < 3; x++) {
            const auto &oh = o.hist_time2(x);
            d.htime2[x].insert(d.htime2[x].end(), oh.begin(), oh.end());
            qsum_fold(d.time2[x], d.qs_time2[x], o.time2[x], o.qs_time2[x]);
            qsum_fold(d.ratio2[x], d.qs_ratio2[x], o.ratio2[x], o.qs_ratio2[x]);
        }
    }
    for (size_t i = 0; i < PV_MIN_WORDS; i++) d.cpc[i] = std::min(d.cpc[i], o.cpc[i]); // CPC union (ICON)
    for (auto &m : o.tops)
        for (auto &kv : m.second) d.tops[m.first][kv.first] += kv.second;
}
} // namespace
extern "C" {

int pv_bucket_merge(pv_ctx *c, uint32_t handler, pv_bucket **bucket, uint32_t period, int prometheus, int merged)
{
    if (!bucket || (handler != PV_HANDLER_NET && handler != PV_HANDLER_DNS)) return c->fail(PV_EINVAL, "bucket merge: one handler");
    std::lock_guard<std::mutex> g(c->mu); // values drained under the lock (pv_window_json)
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    const int part = handler == PV_HANDLER_NET ? PART_NET : PART_DNS;
    const Window &w = part == PART_NET ? c->net : c->dns;
    if (*bucket && (*bucket)->part != part) return c->fail(PV_EINVAL, "bucket merge: a bucket of another handler");
    // StreamMetricsHandler::merge: Prometheus output reads period 1 once the manager holds more
    // than one, never merged
    if (prometheus) { period = w.slots.size() > 1 ? 1 : 0; merged = 0; }
    std::vector<uint32_t> slots;
    if ((rc = window_slots(c, w, period, merged != 0, slots))) return rc;
    HostBucket b;
    // a fresh bucket merged from this handler's bucket(s): CPC through a union (ICON)
    if ((rc = load_bucket(c, slots, true, part, b))) return rc;
    if (!*bucket) {
        pv_bucket *nb = new (std::nothrow) pv_bucket;
        if (!nb) return c->fail(PV_ECAPACITY, "bucket merge: out of host memory");
        nb->part = part;
        nb->handler = handler;
        nb->b = std::move(b);
        *bucket = nb;
        return 0;
    }
    bucket_fold_sum((*bucket)->b, b, part);
    return 0;
}

void pv_bucket_free(pv_bucket *b) { delete b; }

int pv_bucket_json(pv_ctx *c, const pv_bucket *bk, char **out)
{
    *out = nullptr;
    if (!bk) return c->fail(PV_EINVAL, "bucket json: no bucket");
    std::lock_guard<std::mutex> g(c->mu);
    Json j;
    j.obj();
    // window_external_json: {"<schema key>": {period, metrics}} (AbstractMetricsManager.h:589-599)
    // (as pv_window_json: a Net bucket holds the v1 and v2 Net handlers' parts)
    if (bk->part == PART_NET) {
        if (c->net_groups) { j.key("packets").obj(); net_json(c, j, bk->b); j.end_obj(); }
        if (c->net2_groups) { j.key("net").obj(); net2_json(c, j, bk->b); j.end_obj(); }
    } else if (c->dns_groups) {
        j.key("dns").obj();
        if (c->dns2_groups) dns2_json(c, j, bk->b);
        else dns_json(c, j, bk->b);
        j.end_obj();
    }
    j.end_obj();
    *out = strdup(j.s.c_str());
    return 0;
}

int pv_bucket_prometheus(pv_ctx *c, const pv_bucket *bk, const char *const *label_keys, const char *const *label_values,
                         uint32_t n_labels, char **out)
{
    *out = nullptr;
    if (!bk) return c->fail(PV_EINVAL, "bucket prometheus: no bucket");
    std::lock_guard<std::mutex> g(c->mu);
    Prom p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    // window_external_prometheus (AbstractMetricsManager.h:580-587)
    if (bk->part == PART_NET && c->net_groups) {
        net_metrics(c, p, bk->b);
        if (c->net2_groups) net2_metrics(c, p, bk->b);
    }
    if (bk->part == PART_DNS && c->dns_groups) {
        if (c->dns2_groups) dns2_metrics(c, p, bk->b);
        else dns_metrics(c, p, bk->b);
    }
    *out = strdup(p.o.str().c_str());
    return 0;
}

int pv_bucket_opentelemetry(pv_ctx *c, const pv_bucket *bk, const char *const *label_keys, const char *const *label_values,
                            uint32_t n_labels, uint8_t **out, size_t *bytes)
{
    *out = nullptr;
    *bytes = 0;
    if (!bk) return c->fail(PV_EINVAL, "bucket opentelemetry: no bucket");
    std::lock_guard<std::mutex> g(c->mu);
    Otlp p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    // window_external_opentelemetry (AbstractMetricsManager.h:565-578): the bucket's stamps,
    // now for an end it does not have
    p.t0 = (uint64_t)bk->b.start_sec * 1000000000ull + (uint64_t)bk->b.start_nsec;
    if (bk->b.end_sec) p.t1 = (uint64_t)bk->b.end_sec * 1000000000ull + (uint64_t)bk->b.end_nsec;
    else {
        timespec now;
        timespec_get(&now, TIME_UTC);
        p.t1 = (uint64_t)now.tv_sec * 1000000000ull + (uint64_t)now.tv_nsec;
    }
    if (bk->part == PART_NET && c->net_groups) {
        net_metrics(c, p, bk->b);
        if (c->net2_groups) net2_metrics(c, p, bk->b);
    }
    if (bk->part == PART_DNS && c->dns_groups) {
        if (c->dns2_groups) dns2_metrics(c, p, bk->b);
        else dns_metrics(c, p, bk->b);
    }
    *out = (uint8_t *)malloc(p.out.s.size() ? p.out.s.size() : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "bucket opentelemetry: out of host memory");
    memcpy(*out, p.out.s.data(), p.out.s.size());
    *bytes = p.out.s.size();
    return 0;
}

int pv_add_static_label(const char *key, const char *value)
{
    if (!key || !value || !*key) return PV_EINVAL;
    std::lock_guard<std::mutex> g(g_static_mu);
    g_static_labels[key] = value;
    return 0;
}

int pv_window_prometheus(pv_ctx *c, uint32_t period, uint32_t handlers, const char *const *label_keys,
                         const char *const *label_values, uint32_t n_labels, char **out)
{
    *out = nullptr;
    std::lock_guard<std::mutex> g(c->mu); // values drained under the lock (pv_window_json)
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    if (period >= c->cfg.num_periods && period != PV_PERIOD_AUTO)
        return c->fail(PV_EINVAL, "invalid metrics period, specify [0, %u]", c->cfg.num_periods - 1);
    // StreamMetricsHandler::window_prometheus (src/StreamHandler.h:226-233): period 1 of a
    // manager holding more than one bucket, else 0 (each handler's own manager)
    auto per = [&](const Window &w) -> uint32_t { return period != PV_PERIOD_AUTO ? period : (w.slots.size() > 1 ? 1u : 0u); };
    Prom p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    std::vector<uint32_t> slots;
    // each handler's own window (its manager's window_single_prometheus); a handler with
    // every group disabled writes nothing (AbstractMetricsManager.h:522-524)
    if ((handlers & PV_HANDLER_NET) && c->net_groups) {
        if ((rc = window_slots(c, c->net, per(c->net), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_NET, b))) return rc;
        net_metrics(c, p, b);
        if (c->net2_groups) net2_metrics(c, p, b);
    }
    if ((handlers & PV_HANDLER_DNS) && c->dns_groups) {
        if ((rc = window_slots(c, c->dns, per(c->dns), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_DNS, b))) return rc;
        if (c->dns2_groups) dns2_metrics(c, p, b);
        else dns_metrics(c, p, b);
    }
    *out = strdup(p.o.str().c_str());
    return 0;
}

int pv_window_opentelemetry(pv_ctx *c, uint32_t period, uint32_t handlers, const char *const *label_keys,
                            const char *const *label_values, uint32_t n_labels, uint8_t **out, size_t *bytes)
{
    *out = nullptr;
    *bytes = 0;
    std::lock_guard<std::mutex> g(c->mu); // values drained under the lock (pv_window_json)
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    if (period >= c->cfg.num_periods && period != PV_PERIOD_AUTO)
        return c->fail(PV_EINVAL, "invalid metrics period, specify [0, %u]", c->cfg.num_periods - 1);
    // StreamMetricsHandler::window_opentelemetry (src/StreamHandler.h:240-247)
    auto per = [&](const Window &w) -> uint32_t { return period != PV_PERIOD_AUTO ? period : (w.slots.size() > 1 ? 1u : 0u); };
    Otlp p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    std::vector<uint32_t> slots;
    // the bucket's start / end stamps (end unset: now, as window_single_opentelemetry does)
    auto stamps = [&](const Window &w, uint32_t slot) {
        const SlotMeta &m = w.meta[slot];
        p.t0 = (uint64_t)m.start_sec * 1000000000ull + (uint64_t)m.start_nsec;
        if (m.end_sec) p.t1 = (uint64_t)m.end_sec * 1000000000ull + (uint64_t)m.end_nsec;
        else {
            timespec now;
            timespec_get(&now, TIME_UTC);
            p.t1 = (uint64_t)now.tv_sec * 1000000000ull + (uint64_t)now.tv_nsec;
        }
    };
    if ((handlers & PV_HANDLER_NET) && c->net_groups) {
        if ((rc = window_slots(c, c->net, per(c->net), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_NET, b))) return rc;
        stamps(c->net, slots[0]);
        net_metrics(c, p, b);
        if (c->net2_groups) net2_metrics(c, p, b);
    }
    if ((handlers & PV_HANDLER_DNS) && c->dns_groups) {
        if ((rc = window_slots(c, c->dns, per(c->dns), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_DNS, b))) return rc;
        stamps(c->dns, slots[0]);
        if (c->dns2_groups) dns2_metrics(c, p, b);
        else dns_metrics(c, p, b);
    }
    *out = (uint8_t *)malloc(p.out.s.size() ? p.out.s.size() : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "window_opentelemetry: out of host memory");
    memcpy(*out, p.out.s.data(), p.out.s.size());
    *bytes = p.out.s.size();
    return 0;
}

int pv_state_regions(pv_ctx *c, void **sum_ptr, size_t *sum_bytes, void **min_ptr, size_t *min_bytes)
{
    flush_fills(c);
    *sum_ptr = c->d_sum;
    *sum_bytes = (size_t)PV_SLOTS * PV_SUM_WORDS * 8;
    *min_ptr = c->d_cpc;
    *min_bytes = (size_t)PV_SLOTS * PV_MIN_WORDS * 8;
    return 0;
}

// record: u32 table, u64 key, u64 count, u16 name_len, name bytes
int pv_export_topn(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    flush_fills(c);
    std::vector<uint8_t> o;
    std::vector<uint32_t> live; // the tables of both windows
    for (auto s : c->net.slots) live.push_back(s);
    for (auto s : c->dns.slots) live.push_back(s + PV_SLOTS);
    for (uint32_t s : live) {
        std::vector<TopRec> recs;
        int rc = read_topn(c, s, recs);
        if (rc) return rc;
        for (auto &r : recs) {
            uint16_t l = (uint16_t)std::min<size_t>(r.name.size(), 65535);
            size_t p = o.size();
            o.resize(p + 4 + 8 + 8 + 2 + l);
            memcpy(&o[p], &s, 4);
            memcpy(&o[p + 4], &r.key, 8);
            memcpy(&o[p + 12], &r.count, 8);
            memcpy(&o[p + 20], &l, 2);
            memcpy(&o[p + 22], r.name.data(), l);
        }
    }
    *bytes = o.size();
    *buf = (uint8_t *)malloc(o.size() ? o.size() : 1);
    if (!o.empty()) memcpy(*buf, o.data(), o.size());
    return 0;
}

int pv_merge_topn(pv_ctx *c, const uint8_t *buf, size_t bytes)
{
    mark_merged(c, "pv_merge_topn");
    size_t p = 0;
    while (p + 22 <= bytes) {
        uint32_t s; uint64_t key, cnt; uint16_t l;
        memcpy(&s, buf + p, 4); memcpy(&key, buf + p + 4, 8); memcpy(&cnt, buf + p + 12, 8); memcpy(&l, buf + p + 20, 2);
        if (p + 22 + l > bytes || s >= PV_TABLES) return c->fail(PV_EINVAL, "malformed top-N buffer");
        auto &e = c->remote_topn[s][key];
        e.first += cnt;
        e.second.assign((const char *)buf + p + 22, l);
        p += 22 + l;
    }
    return 0;
}

int comm_allgather_locked(pv_ctx *c, const void *buf, size_t bytes, std::vector<uint8_t> &out);

// ------------------------------------------------------------------ multi-GPU top-N exchange
// (pv_topn_x_*, pv_comm_merge_topn; kernels pv_topn_x* in pv_kernels.hip). Every table's
// regions are split over the ranks in contiguous blocks; a rank ships the live entries of the
// regions others own to their owners (device lists, RCCL point-to-point or host blobs), and
// each owner merges them into its regions with pv_topn_merge. Afterwards a rank's top-N view is
// its own regions; pv_topn_x_candidates / _names / _view then assemble the merged lists from
// every owner's leading entries, names fetched from whichever rank holds them.
namespace {
const uint32_t X_MAGIC = 0x31585650u; // "PVX1"
// candidates per metric and owner: topn_count and the entries tied with the last; a tied group
// larger than this is cut by key order (the merged list's order among equal estimates can then
// differ from one stream's, which orders them by name)
const size_t PV_X_TIES = 8192;
struct XPrep {
    PvXTabs T;
    uint32_t nreg = 0, E = 0;
    std::vector<uint32_t> hdr;      // the header stream, (owner, handler, region, slot) order
    std::vector<uint64_t> dtot, dstart; // entries per owner, where its slice starts
};
uint32_t x_lo_h(uint32_t d, uint32_t nreg, uint32_t W) { return (uint32_t)(((uint64_t)d * nreg + W - 1) / W); }

void x_tables(pv_ctx *c, PvXTabs &T, uint32_t W, uint32_t me)
{
    memset(&T, 0, sizeof T);
    T.W = W;
    T.me = me;
    for (uint32_t s : c->net.slots) T.tb[T.n++] = s;
    for (uint32_t s : c->dns.slots) T.tb[T.n++] = PV_SLOTS + s;
}

// the parameter block the exchange kernels read (tables, geometry), uploaded to d_xp
int x_params(pv_ctx *c, PvParams &P)
{
    params_common(c, P, nullptr, nullptr, 0);
    P.tcap_log2 = c->tcap_log2;
    P.reg_log2 = c->reg_log2;
    P.tkeys = c->d_tkeys;
    P.tcnt = c->d_tcnt;
    P.taux = c->d_taux;
    P.tab_live = c->d_tab_live;
    P.flags = c->d_status + ST_FLAGS;
    P.cpc = c->d_cpc;
    P.sum = c->d_sum;
    hipError_t e;
    if (!c->d_xp && !hip_ok(e = hipMalloc(&c->d_xp, sizeof(PvParams)))) return c->hipfail(e, "exchange parameters");
    if (!hip_ok(e = hipMemcpyAsync(c->d_xp, &P, sizeof P, hipMemcpyHostToDevice, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange parameters");
    return 0;
}

int x_grow(pv_ctx *c, void **p, size_t &have, size_t need, const char *what)
{
    if (need <= have) return 0;
    hipError_t e;
    if (*p) hipFree(*p);
    *p = nullptr;
    have = 0;
    if (!hip_ok(e = hipMalloc(p, std::max<size_t>(need, 256)))) return c->hipfail(e, what);
    have = std::max<size_t>(need, 256);
    return 0;
}

// the send list on the device (d_xsend) and its layout on the host
int x_prepare(pv_ctx *c, uint32_t W, uint32_t me, XPrep &X)
{
    hipSetDevice(c->device);
    flush_fills(c);
    x_tables(c, X.T, W, me);
    X.nreg = 1u << c->reg_log2;
    X.E = 2 * X.nreg * PV_SLOTS;
    PvParams P;
    if (int rc = x_params(c, P)) return rc;
    hipError_t e;
    size_t need = (size_t)X.E * 4;
    if (int rc = x_grow(c, (void **)&c->d_xcnt, c->xcnt_bytes, need * 3, "exchange counts")) return rc;
    uint32_t *d_cnt = c->d_xcnt, *d_off = c->d_xcnt + X.E, *d_hdr = c->d_xcnt + 2 * X.E;
    if (!hip_ok(e = hipMemsetAsync(d_cnt, 0, need, c->stream))) return c->hipfail(e, "exchange counts");
    if (X.T.n) {
        hipLaunchKernelGGL(pv_topn_xcount, dim3(X.T.n * X.nreg), dim3(256), 0, c->stream, (const PvParams *)c->d_xp, X.T, d_cnt);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_topn_xcount");
    }
    hipLaunchKernelGGL(pv_topn_xscan, dim3(1), dim3(1024), 0, c->stream, c->reg_log2, W, (const uint32_t *)d_cnt, d_off, d_hdr);
    X.hdr.resize(X.E);
    if (!hip_ok(e = hipGetLastError()) ||
        !hip_ok(e = hipMemcpyAsync(X.hdr.data(), d_hdr, need, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange scan");
    X.dtot.assign(W, 0);
    X.dstart.assign(W + 1, 0);
    for (uint32_t d = 0; d < W; d++) {
        const uint32_t lo = x_lo_h(d, X.nreg, W), hi = x_lo_h(d + 1, X.nreg, W);
        for (uint32_t p = 2 * PV_SLOTS * lo; p < 2 * PV_SLOTS * hi; p++) X.dtot[d] += X.hdr[p];
        X.dstart[d + 1] = X.dstart[d] + X.dtot[d];
    }
    if (int rc = x_grow(c, &c->d_xsend, c->xsend_bytes, (size_t)X.dstart[W] * 16, "exchange send list")) return rc;
    if (X.T.n && X.dstart[W]) {
        hipLaunchKernelGGL(pv_topn_xwrite, dim3(X.T.n * X.nreg), dim3(256), 0, c->stream, (const PvParams *)c->d_xp, X.T,
                           (const uint32_t *)d_off, (ulonglong2 *)c->d_xsend);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "exchange list");
    }
    return 0;
}

// merge the received lists (device: d_xrecv, W slots of `stride` entries; headers d_xrhdr) into
// this rank's regions
int x_merge_recv(pv_ctx *c, uint32_t W, uint32_t me, const std::vector<uint64_t> &rtot, uint64_t stride)
{
    const uint32_t nreg = 1u << c->reg_log2;
    const uint32_t lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    if (stride >= (1u << 24)) return c->fail(PV_ECAPACITY, "multi-GPU top-N exchange: %lu entries from one rank exceed 2^24",
                                             (unsigned long)stride);
    uint64_t total = 0;
    for (uint64_t v : rtot) total += v;
    hipError_t e;
    // the run table ([run key][column] of W columns, pv_topn_merge's layout)
    if (W > c->cb_h_grid) {
        if (c->d_cb_h) hipFree(c->d_cb_h);
        c->d_cb_h = nullptr;
        c->cb_h_grid = 0;
        if (!hip_ok(e = hipMalloc(&c->d_cb_h, (size_t)((W + 7) & ~7u) << (PV_MAX_REGIONS_LOG2 + 4)))) return c->hipfail(e, "region runs");
        c->cb_h_grid = W;
    }
    if (!total) { c->x_ranks = W; c->x_rank = me; return 0; }
    hipLaunchKernelGGL(pv_topn_xruns, dim3(W), dim3(1024), 0, c->stream, c->reg_log2, W, me, (const uint32_t *)c->d_xrhdr,
                       2 * PV_SLOTS * (hi - lo), (uint64_t *)c->d_cb_h);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_topn_xruns");
    PvParams P;
    params_common(c, P, nullptr, nullptr, 0);
    P.tcap_log2 = c->tcap_log2;
    P.reg_log2 = c->reg_log2;
    P.tkeys = c->d_tkeys;
    P.tcnt = c->d_tcnt;
    P.taux = c->d_taux;
    P.tab_live = c->d_tab_live;
    P.flags = c->d_status + ST_FLAGS;
    P.cpc = c->d_cpc;
    P.xmerge = 1;
    P.x_lo = lo;
    P.x_hi = hi;
    // a full region's entries go to the overflow list; the table is purged (the frequent-items
    // merge's purge, src/Metrics.h:534-538) and they are inserted again (drain_overflow)
    P.ovf = c->d_ovf;
    P.ovf_cnt = c->d_ovf_cnt;
    P.ovf_cap = c->ovf_cap;
    P.arena = c->d_arena;
    P.arena_top = c->d_arena_top;
    P.arena_cap = c->arena_cap;
    P.cb = (uint64_t *)c->d_xrecv;
    P.cb_fan = 1;
    P.mq_cap = (uint32_t)stride;
    P.cb_grid = W;
    P.cb_run = (uint64_t *)c->d_cb_h;
    P.cb_hm = c->d_cb_cnt + 32768;
    P.tp_hands = c->d_cb_cnt + 32768 + 1024; // a word holding 3: both handlers
    P.slot_of[0] = c->net.slots.empty() ? 0 : c->net.slots.front();
    P.dslot_of[0] = c->dns.slots.empty() ? 0 : c->dns.slots.front();
    if (W + 1 > 1024 + 1) return c->fail(PV_EINVAL, "%u ranks", W);
    launch_fill32(c, c->d_cb_cnt + 32768, 1024 + 1, 3u);
    launch_fill32(c, c->d_status + ST_FLAGS, 1, 0u);
    flush_fills(c);
    if (!c->d_xp && !hip_ok(e = hipMalloc(&c->d_xp, sizeof(PvParams)))) return c->hipfail(e, "exchange parameters");
    if (!hip_ok(e = hipMemcpyAsync(c->d_xp, &P, sizeof P, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "exchange parameters");
    hipLaunchKernelGGL(pv_topn_merge, dim3(2u << c->reg_log2), dim3(pv_topn_merge_threads()), 0, c->stream, (const PvParams *)c->d_xp);
    uint32_t flags = 0;
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "exchange merge");
    if (int rc = drain_overflow(c, c->stream, false, nullptr, c->d_xp)) return rc;
    if (!hip_ok(e = hipMemcpyAsync(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange merge");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "multi-GPU top-N merge: the overflow list is full (raise table_log2)");
    for (uint32_t s : c->net.slots) c->net.clean[s] = false;
    for (uint32_t s : c->dns.slots) c->dns.clean[s] = false;
    c->x_ranks = W;
    c->x_rank = me;
    return 0;
}

// the purge offsets (frequent-items thetas) of the live tables' regions, nreg u64 per table
void x_roff_pack(pv_ctx *c, const PvXTabs &T, uint32_t nreg, std::vector<uint64_t> &o)
{
    o.assign((size_t)T.n * nreg, 0);
    for (uint32_t t = 0; t < T.n; t++)
        if (!c->roff[T.tb[t]].empty())
            for (uint32_t r = 0; r < nreg; r++) o[(size_t)t * nreg + r] = c->roff[T.tb[t]][r];
}
// add another rank's offsets of this rank's regions
void x_roff_add(pv_ctx *c, const PvXTabs &T, uint32_t nreg, uint32_t lo, uint32_t hi, const uint64_t *o)
{
    for (uint32_t t = 0; t < T.n; t++) {
        bool any = false;
        for (uint32_t r = lo; r < hi && !any; r++) any = o[(size_t)t * nreg + r] != 0;
        if (!any) continue;
        std::vector<uint64_t> &ro = c->roff[T.tb[t]];
        if (ro.empty()) ro.assign(nreg, 0);
        for (uint32_t r = lo; r < hi; r++) ro[r] += o[(size_t)t * nreg + r];
    }
}
} // namespace

// blob: magic, W, rank, ntab, nreg | tb[ntab] | roff[ntab][nreg] | dtot[W] | hdr[E] | entries
int pv_topn_x_export(pv_ctx *c, uint32_t W, uint32_t me, uint8_t **blob, size_t *bytes)
{
    *blob = nullptr;
    *bytes = 0;
    if (W < 1 || me >= W || W > 1024) return c->fail(PV_EINVAL, "rank %u of %u", me, W);
    std::lock_guard<std::mutex> g(c->mu);
    XPrep X;
    if (int rc = x_prepare(c, W, me, X)) return rc;
    std::vector<uint64_t> ro;
    x_roff_pack(c, X.T, X.nreg, ro);
    const size_t head = 20 + 4 * (size_t)X.T.n;
    const size_t n = head + ro.size() * 8 + (size_t)W * 8 + (size_t)X.E * 4 + (size_t)X.dstart[W] * 16;
    uint8_t *o = (uint8_t *)malloc(n);
    if (!o) return c->fail(PV_ECAPACITY, "exchange blob");
    const uint32_t h[5] = {X_MAGIC, W, me, X.T.n, X.nreg};
    memcpy(o, h, 20);
    memcpy(o + 20, X.T.tb, 4 * (size_t)X.T.n);
    size_t at = head;
    memcpy(o + at, ro.data(), ro.size() * 8);
    at += ro.size() * 8;
    memcpy(o + at, X.dtot.data(), (size_t)W * 8);
    at += (size_t)W * 8;
    memcpy(o + at, X.hdr.data(), (size_t)X.E * 4);
    at += (size_t)X.E * 4;
    hipError_t e;
    if (X.dstart[W] && !hip_ok(e = hipMemcpy(o + at, c->d_xsend, (size_t)X.dstart[W] * 16, hipMemcpyDeviceToHost))) {
        free(o);
        return c->hipfail(e, "exchange download");
    }
    *blob = o;
    *bytes = n;
    return 0;
}

int pv_topn_x_import(pv_ctx *c, uint32_t W, uint32_t me, const uint8_t *const *blobs, const size_t *sizes)
{
    mark_merged(c, "pv_topn_x_import");
    if (W < 1 || me >= W || W > 1024) return c->fail(PV_EINVAL, "rank %u of %u", me, W);
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    PvXTabs T;
    x_tables(c, T, W, me);
    const uint32_t nreg = 1u << c->reg_log2, E = 2 * nreg * PV_SLOTS;
    const uint32_t lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    struct Src { const uint64_t *ro, *dtot; const uint32_t *hdr; const uint8_t *ent; };
    std::vector<Src> src(W);
    std::vector<uint64_t> rtot(W, 0);
    uint64_t stride = 0;
    for (uint32_t q = 0; q < W; q++) {
        const uint8_t *b = blobs[q];
        uint32_t h[5];
        if (!b || sizes[q] < 20) return c->fail(PV_EINVAL, "exchange blob %u missing", q);
        memcpy(h, b, 20);
        if (h[0] != X_MAGIC || h[1] != W || h[2] != q || h[3] != T.n || h[4] != nreg || memcmp(b + 20, T.tb, 4 * (size_t)T.n))
            return c->fail(PV_EINVAL, "exchange blob %u does not match this rank's windows", q);
        size_t at = 20 + 4 * (size_t)T.n;
        // the fixed sections (region offsets, per-owner totals, counts) must lie in the blob
        // before any of them is read
        if (at + (size_t)T.n * nreg * 8 + (size_t)W * 8 + (size_t)E * 4 > sizes[q])
            return c->fail(PV_EINVAL, "exchange blob %u truncated", q);
        src[q].ro = reinterpret_cast<const uint64_t *>(b + at);
        at += (size_t)T.n * nreg * 8;
        src[q].dtot = reinterpret_cast<const uint64_t *>(b + at);
        at += (size_t)W * 8;
        src[q].hdr = reinterpret_cast<const uint32_t *>(b + at);
        at += (size_t)E * 4;
        src[q].ent = b + at;
        uint64_t all = 0;
        for (uint32_t d = 0; d < W; d++) {
            if (src[q].dtot[d] > (uint64_t)1 << 40) return c->fail(PV_EINVAL, "exchange blob %u: bad entry total", q);
            all += src[q].dtot[d];
        }
        if (at + all * 16 > sizes[q]) return c->fail(PV_EINVAL, "exchange blob %u truncated", q);
        // the counts of this rank's slice (owner me: cells [2 * PV_SLOTS * lo, 2 * PV_SLOTS * hi))
        // index the receive list on the device (pv_topn_xruns / pv_topn_merge): they must add up to
        // what the source sends this rank
        uint64_t mine = 0;
        for (size_t k = (size_t)2 * PV_SLOTS * lo; k < (size_t)2 * PV_SLOTS * hi; k++) mine += src[q].hdr[k];
        if (mine != src[q].dtot[me]) return c->fail(PV_EINVAL, "exchange blob %u: counts do not match its total", q);
        rtot[q] = q == me ? 0 : src[q].dtot[me];
        stride = std::max(stride, rtot[q]);
    }
    hipError_t e;
    const size_t hlen = (size_t)2 * PV_SLOTS * (hi - lo);
    if (int rc = x_grow(c, (void **)&c->d_xrhdr, c->xrhdr_bytes, std::max<size_t>(1, W * hlen) * 4, "exchange headers")) return rc;
    if (int rc = x_grow(c, &c->d_xrecv, c->xrecv_bytes, std::max<size_t>(1, W * stride) * 16, "exchange receive list")) return rc;
    for (uint32_t q = 0; q < W; q++) {
        if (q == me) continue;
        uint64_t before = 0;
        for (uint32_t d = 0; d < me; d++) before += src[q].dtot[d];
        if (!hip_ok(e = hipMemcpyAsync(c->d_xrhdr + (size_t)q * hlen, src[q].hdr + (size_t)2 * PV_SLOTS * lo, hlen * 4,
                                       hipMemcpyHostToDevice, c->stream)) ||
            (rtot[q] && !hip_ok(e = hipMemcpyAsync((uint8_t *)c->d_xrecv + (size_t)q * stride * 16, src[q].ent + before * 16,
                                                   rtot[q] * 16, hipMemcpyHostToDevice, c->stream))))
            return c->hipfail(e, "exchange upload");
        x_roff_add(c, T, nreg, lo, hi, src[q].ro);
    }
    return x_merge_recv(c, W, me, rtot, stride);
}

int pv_comm_merge_topn(pv_ctx *c)
{
    mark_merged(c, "pv_comm_merge_topn");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    const uint32_t W = (uint32_t)c->comm_ranks, me = (uint32_t)c->comm_rank;
    std::lock_guard<std::mutex> g(c->mu);
    XPrep X;
    if (int rc = x_prepare(c, W, me, X)) return rc;
    const uint32_t nreg = X.nreg, lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    hipError_t e;
    // entries per (source, this rank), and the purge offsets: one small all-to-all / all-gather
    if (int rc = x_grow(c, (void **)&c->d_xtot, c->xtot_bytes, (size_t)W * 16, "exchange counts")) return rc;
    if (!hip_ok(e = hipMemcpyAsync(c->d_xtot, X.dtot.data(), (size_t)W * 8, hipMemcpyHostToDevice, c->stream)))
        return c->hipfail(e, "exchange counts");
    ncclResult_t r = ncclGroupStart();
    for (uint32_t q = 0; q < W && r == ncclSuccess; q++) {
        if (q == me) continue;
        r = ncclSend(c->d_xtot + q, 1, ncclUint64, (int)q, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->d_xtot + W + q, 1, ncclUint64, (int)q, c->comm, c->stream);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) return c->fail(PV_EHIP, "exchange counts: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    std::vector<uint64_t> rtot(W, 0);
    if (!hip_ok(e = hipMemcpyAsync(rtot.data(), c->d_xtot + W, (size_t)W * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange counts");
    rtot[me] = 0;
    uint64_t stride = 0;
    for (uint64_t v : rtot) stride = std::max(stride, v);
    const size_t hlen = (size_t)2 * PV_SLOTS * (hi - lo);
    if (int rc = x_grow(c, (void **)&c->d_xrhdr, c->xrhdr_bytes, std::max<size_t>(1, W * hlen) * 4, "exchange headers")) return rc;
    if (int rc = x_grow(c, &c->d_xrecv, c->xrecv_bytes, std::max<size_t>(1, W * stride) * 16, "exchange receive list")) return rc;
    const uint32_t *d_hdr = c->d_xcnt + 2 * X.E;
    r = ncclGroupStart();
    for (uint32_t q = 0; q < W && r == ncclSuccess; q++) {
        if (q == me) continue;
        const uint32_t qlo = x_lo_h(q, nreg, W), qhi = x_lo_h(q + 1, nreg, W);
        r = ncclSend(d_hdr + (size_t)2 * PV_SLOTS * qlo, (size_t)2 * PV_SLOTS * (qhi - qlo), ncclUint32, (int)q, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->d_xrhdr + (size_t)q * hlen, hlen, ncclUint32, (int)q, c->comm, c->stream);
        if (r == ncclSuccess && X.dtot[q])
            r = ncclSend((const uint8_t *)c->d_xsend + X.dstart[q] * 16, X.dtot[q] * 2, ncclUint64, (int)q, c->comm, c->stream);
        if (r == ncclSuccess && rtot[q])
            r = ncclRecv((uint8_t *)c->d_xrecv + (size_t)q * stride * 16, rtot[q] * 2, ncclUint64, (int)q, c->comm, c->stream);
    }
    r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) return c->fail(PV_EHIP, "exchange lists: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    // purge offsets (host blobs, a few KB)
    {
        std::vector<uint64_t> ro;
        x_roff_pack(c, X.T, nreg, ro);
        bool any = false;
        for (uint64_t v : ro) any |= v != 0;
        uint8_t anyb = any ? 1 : 0;
        // (skipped when no rank purged: one byte each first)
        std::vector<uint8_t> flags;
        if (int rc = comm_allgather_locked(c, &anyb, 1, flags)) return rc;
        bool someone = false;
        for (uint8_t f : flags) someone |= f != 0;
        if (someone) {
            std::vector<uint8_t> all;
            if (int rc = comm_allgather_locked(c, ro.data(), ro.size() * 8, all)) return rc;
            for (uint32_t q = 0; q < W; q++)
                if (q != me) x_roff_add(c, X.T, nreg, lo, hi, reinterpret_cast<const uint64_t *>(all.data() + (size_t)q * ro.size() * 8));
        }
    }
    return x_merge_recv(c, W, me, rtot, stride);
}

// ---- the merged view's lists: every owner's leading entries per metric, names from any rank
namespace {
// the text of a table entry's name record (read_topn's rules)
void x_name_text(uint32_t metric, const uint8_t *rec, uint32_t len, std::string &out)
{
    char b[64];
    if (metric == TM_IPV6 && len == 16) out = inet_ntop(AF_INET6, rec, b, sizeof b) ? b : "";
    else if (metric == TM_ECS && len == 17) out = inet_ntop(rec[0] == 1 ? AF_INET : AF_INET6, rec + 1, b, sizeof b) ? b : "";
    else out.assign((const char *)rec, len);
}
// the texts of many name records at once (pv_xname_len / pv_xname_copy): ok[i] false where aux[i]
// is 0 (no record)
int x_read_names(pv_ctx *c, const std::vector<uint32_t> &tb, const std::vector<uint32_t> &aux, const std::vector<uint64_t> &key,
                 std::vector<std::string> &out, std::vector<bool> &ok)
{
    const size_t n = tb.size();
    out.assign(n, std::string());
    ok.assign(n, false);
    if (!n) return 0;
    hipError_t e;
    uint32_t *d_tb = nullptr, *d_aux = nullptr, *d_len = nullptr;
    uint64_t *d_off = nullptr;
    uint8_t *d_out = nullptr;
    struct Free { void *p[5]; ~Free() { for (void *q : p) if (q) hipFree(q); } } fr{{nullptr, nullptr, nullptr, nullptr, nullptr}};
    if (!hip_ok(e = hipMalloc(&d_tb, n * 4)) || !hip_ok(e = hipMalloc(&d_aux, n * 4)) || !hip_ok(e = hipMalloc(&d_len, n * 4)) ||
        !hip_ok(e = hipMalloc(&d_off, n * 8)))
        return c->hipfail(e, "name gather");
    fr.p[0] = d_tb; fr.p[1] = d_aux; fr.p[2] = d_len; fr.p[3] = d_off;
    std::vector<uint32_t> len(n);
    const uint32_t g = (uint32_t)((n + 255) / 256);
    if (!hip_ok(e = hipMemcpyAsync(d_tb, tb.data(), n * 4, hipMemcpyHostToDevice, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(d_aux, aux.data(), n * 4, hipMemcpyHostToDevice, c->stream)))
        return c->hipfail(e, "name gather");
    hipLaunchKernelGGL(pv_xname_len, dim3(g), dim3(256), 0, c->stream, c->d_arena, c->arena_cap, d_tb, d_aux, (uint32_t)n, d_len);
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(len.data(), d_len, n * 4, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "name gather");
    std::vector<uint64_t> off(n);
    uint64_t tot = 0;
    for (size_t i = 0; i < n; i++) { off[i] = tot; tot += len[i] == 0xffffffffu ? 0 : len[i]; }
    std::vector<uint8_t> bytes(tot);
    if (tot) {
        if (!hip_ok(e = hipMalloc(&d_out, tot))) return c->hipfail(e, "name gather");
        fr.p[4] = d_out;
        if (!hip_ok(e = hipMemcpyAsync(d_off, off.data(), n * 8, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "name gather");
        hipLaunchKernelGGL(pv_xname_copy, dim3(g), dim3(256), 0, c->stream, c->d_arena, c->arena_cap, d_tb, d_aux, d_len, d_off,
                           (uint32_t)n, d_out);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(bytes.data(), d_out, tot, hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "name gather");
    }
    for (size_t i = 0; i < n; i++) {
        if (len[i] == 0xffffffffu) continue;
        x_name_text(PV_KEY_METRIC(key[i]), bytes.data() + off[i], len[i], out[i]);
        ok[i] = true;
    }
    return 0;
}
void put_u32(std::vector<uint8_t> &o, uint32_t v) { const size_t p = o.size(); o.resize(p + 4); memcpy(&o[p], &v, 4); }
void put_u64(std::vector<uint8_t> &o, uint64_t v) { const size_t p = o.size(); o.resize(p + 8); memcpy(&o[p], &v, 8); }
void put_name(std::vector<uint8_t> &o, const std::string *s)
{
    const uint16_t l = s ? (uint16_t)std::min<size_t>(s->size(), 65534) : (uint16_t)0xffff;
    const size_t p = o.size();
    o.resize(p + 2 + (s ? l : 0));
    memcpy(&o[p], &l, 2);
    if (s && l) memcpy(&o[p + 2], s->data(), l);
}
} // namespace

// The slot sets a window read asks for, per part: each live slot alone and each run of the most
// recent slots (merged windows); a set id is part << 16 | slot mask.
void x_slot_sets(pv_ctx *c, int part, std::vector<uint32_t> &v)
{
    const Window &w = part == PART_NET ? c->net : c->dns;
    v.clear();
    uint32_t m = 0;
    for (size_t i = 0; i < w.slots.size(); i++) {
        v.push_back(((uint32_t)part << 16) | (1u << w.slots[i]));
        m |= 1u << w.slots[i];
        if (i) v.push_back(((uint32_t)part << 16) | m);
    }
}

// candidates: u32 set id | u64 key | u64 estimate | u16 name length (0xffff: unknown here) | name.
// Per slot set and metric, this rank's regions' leading entries by the estimate summed over the
// set's tables (the merged window's counts).
int pv_topn_x_candidates(pv_ctx *c, uint8_t **blob, size_t *bytes)
{
    *blob = nullptr;
    *bytes = 0;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->x_ranks < 1) return c->fail(PV_EINVAL, "no multi-GPU top-N merge on this context (pv_topn_x_import / pv_comm_merge_topn)");
    hipSetDevice(c->device);
    flush_fills(c);
    const uint32_t W = c->x_ranks, me = c->x_rank, nreg = 1u << c->reg_log2, rsl = c->tcap_log2 - c->reg_log2;
    const uint32_t lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    const size_t K = std::max<size_t>(c->cfg.topn_count, 1);
    const size_t n = (size_t)(hi - lo) << rsl;
    std::vector<uint8_t> o;
    hipError_t e;
    // each live table's regions, read once
    struct Slice { std::vector<uint64_t> keys, cnt; std::vector<uint32_t> aux; };
    std::map<uint32_t, Slice> sl;
    auto slice = [&](uint32_t tb) -> const Slice * {
        auto it = sl.find(tb);
        if (it != sl.end()) return &it->second;
        Slice &x = sl[tb];
        const size_t base = ((size_t)tb << c->tcap_log2) + ((size_t)lo << rsl);
        x.keys.resize(n); x.cnt.resize(n); x.aux.resize(n);
        if (n && (!hip_ok(e = hipMemcpy(x.keys.data(), c->d_tkeys + base, n * 8, hipMemcpyDeviceToHost)) ||
                  !hip_ok(e = hipMemcpy(x.cnt.data(), c->d_tcnt + base, n * 8, hipMemcpyDeviceToHost)) ||
                  !hip_ok(e = hipMemcpy(x.aux.data(), c->d_taux + base, n * 4, hipMemcpyDeviceToHost))))
            return nullptr;
        return &x;
    };
    // Per part: every live slot's entries of this rank's regions, sorted by key once; then per key
    // its estimate in each slot set (single slots and the merged runs) and, per (set, metric), the
    // topn_count leading entries with the ties of the last: a first walk finds each list's
    // threshold (a bounded heap of estimates), a second collects the entries at or above it.
    struct XE { uint64_t key, est; uint32_t tb, aux; uint32_t slot; };
    struct XOut { uint32_t set; uint64_t key, est; uint32_t tb, aux; };
    std::vector<XOut> out;
    for (int part = PART_NET; part <= PART_DNS; part++) {
        std::vector<uint32_t> sets;
        x_slot_sets(c, part, sets);
        if (sets.empty()) continue;
        const Window &w = part == PART_NET ? c->net : c->dns;
        std::vector<XE> ents;
        for (uint32_t s : w.slots) {
            const uint32_t tb = s + (part == PART_DNS ? PV_SLOTS : 0);
            const Slice *x = slice(tb);
            if (!x) return c->hipfail(e, "read top-N regions");
            const std::vector<uint64_t> &roff = c->roff[tb];
            for (size_t i = 0; i < n; i++)
                if (x->keys[i])
                    ents.push_back(XE{x->keys[i], x->cnt[i] + (roff.empty() ? 0 : roff[lo + (i >> rsl)]), tb, x->aux[i], s});
        }
        std::sort(ents.begin(), ents.end(), [](const XE &p1, const XE &p2) { return p1.key < p2.key; });
        const size_t NZ = sets.size();
        // per key group [g0, g1): the estimate in set z, and whether the set holds the key
        auto group_est = [&](size_t g0, size_t g1, size_t z, uint64_t &est) {
            bool in = false;
            est = 0;
            for (size_t j = g0; j < g1; j++)
                if ((sets[z] >> ents[j].slot) & 1) { est += ents[j].est; in = true; }
            return in;
        };
        // walk 1: thresholds (a min-heap of the K largest estimates per (set, metric))
        std::map<std::pair<uint32_t, uint32_t>, std::priority_queue<uint64_t, std::vector<uint64_t>, std::greater<uint64_t>>> heaps;
        for (size_t g0 = 0, g1; g0 < ents.size(); g0 = g1) {
            g1 = g0 + 1;
            while (g1 < ents.size() && ents[g1].key == ents[g0].key) g1++;
            const uint32_t hm = host_metric(c, ents[g0].key);
            for (size_t z = 0; z < NZ; z++) {
                uint64_t est;
                if (!group_est(g0, g1, z, est)) continue;
                auto &h = heaps[{(uint32_t)z, hm}];
                if (h.size() < K) h.push(est);
                else if (est > h.top()) { h.pop(); h.push(est); }
            }
        }
        std::map<std::pair<uint32_t, uint32_t>, uint64_t> thr;
        for (auto &kv : heaps) thr[kv.first] = kv.second.size() < K ? 0 : kv.second.top();
        // walk 2: entries at or above the threshold (est, key, name table, name aux)
        std::map<std::pair<uint32_t, uint32_t>, std::vector<std::tuple<uint64_t, uint64_t, uint32_t, uint32_t>>> got;
        for (size_t g0 = 0, g1; g0 < ents.size(); g0 = g1) {
            g1 = g0 + 1;
            while (g1 < ents.size() && ents[g1].key == ents[g0].key) g1++;
            const uint32_t hm = host_metric(c, ents[g0].key);
            for (size_t z = 0; z < NZ; z++) {
                uint64_t est;
                if (!group_est(g0, g1, z, est)) continue;
                if (est < thr[{(uint32_t)z, hm}]) continue;
                uint32_t ntb = 0, naux = 0;
                for (size_t j = g0; j < g1 && !naux; j++)
                    if (((sets[z] >> ents[j].slot) & 1) && ents[j].aux) { ntb = ents[j].tb; naux = ents[j].aux; }
                auto &v = got[{(uint32_t)z, hm}];
                v.emplace_back(est, ents[g0].key, ntb, naux);
                if (v.size() > 4 * (PV_X_TIES + K)) {
                    // a flat list: keep the leading ones by (estimate desc, key asc)
                    auto cmp = [](const auto &a1, const auto &b1) {
                        return std::get<0>(a1) != std::get<0>(b1) ? std::get<0>(a1) > std::get<0>(b1) : std::get<1>(a1) < std::get<1>(b1);
                    };
                    std::nth_element(v.begin(), v.begin() + (PV_X_TIES + K), v.end(), cmp);
                    v.resize(PV_X_TIES + K);
                }
            }
        }
        for (size_t z = 0; z < NZ; z++) {
            for (auto it = got.lower_bound({(uint32_t)z, 0u}); it != got.end() && it->first.first == z; ++it) {
                auto &v = it->second;
                std::sort(v.begin(), v.end(), [](const auto &a1, const auto &b1) {
                    return std::get<0>(a1) != std::get<0>(b1) ? std::get<0>(a1) > std::get<0>(b1) : std::get<1>(a1) < std::get<1>(b1);
                });
                // the topn_count leading entries and every entry tied with the last of them (the lists
                // order ties by name, which only the whole tied group decides; at most PV_X_TIES)
                size_t m = std::min(K, v.size());
                while (m < v.size() && m < PV_X_TIES && std::get<0>(v[m]) == std::get<0>(v[m - 1])) m++;
                for (size_t k = 0; k < m; k++) out.push_back(XOut{sets[z], std::get<1>(v[k]), std::get<0>(v[k]), std::get<2>(v[k]), std::get<3>(v[k])});
            }
        }
    }
    // the names: IPv4 from the key, the others gathered from the arena in one pass
    {
        std::vector<uint32_t> gtb, gaux;
        std::vector<uint64_t> gkey;
        std::vector<size_t> at;
        for (size_t i = 0; i < out.size(); i++)
            if (PV_KEY_METRIC(out[i].key) != TM_IPV4 && out[i].aux) {
                gtb.push_back(out[i].tb); gaux.push_back(out[i].aux); gkey.push_back(out[i].key); at.push_back(i);
            }
        std::vector<std::string> txt;
        std::vector<bool> okv;
        if (int rc = x_read_names(c, gtb, gaux, gkey, txt, okv)) return rc;
        std::vector<const std::string *> nmp(out.size(), nullptr);
        for (size_t j = 0; j < at.size(); j++) if (okv[j]) nmp[at[j]] = &txt[j];
        for (size_t i = 0; i < out.size(); i++) {
            const uint64_t key = out[i].key;
            put_u32(o, out[i].set);
            put_u64(o, key);
            put_u64(o, out[i].est);
            if (PV_KEY_METRIC(key) == TM_IPV4) {
                const uint32_t ip = (uint32_t)key;
                char bb[20];
                snprintf(bb, sizeof bb, "%u.%u.%u.%u", ip & 0xff, (ip >> 8) & 0xff, (ip >> 16) & 0xff, ip >> 24);
                const std::string nm = bb;
                put_name(o, &nm);
            } else {
                put_name(o, nmp[i]);
            }
        }
    }
    *blob = (uint8_t *)malloc(std::max<size_t>(o.size(), 1));
    if (!*blob) return c->fail(PV_ECAPACITY, "candidates");
    memcpy(*blob, o.data(), o.size());
    *bytes = o.size();
    return 0;
}

namespace {
struct XCand {
    uint32_t tb;
    uint64_t key, est;
    bool named;
    std::string name;
};
bool x_parse_cands(const uint8_t *b, size_t n, std::vector<XCand> &out)
{
    size_t p = 0;
    while (p < n) {
        if (p + 22 > n) return false;
        XCand x;
        uint16_t l;
        memcpy(&x.tb, b + p, 4);
        memcpy(&x.key, b + p + 4, 8);
        memcpy(&x.est, b + p + 12, 8);
        memcpy(&l, b + p + 20, 2);
        p += 22;
        x.named = l != 0xffff;
        if (x.named) {
            if (p + l > n) return false;
            x.name.assign((const char *)b + p, l);
            p += l;
        }
        out.push_back(std::move(x));
    }
    return true;
}
} // namespace

// answers: the names this rank holds for candidates (of every rank) that came without one:
// u32 tb | u64 key | u16 length | name
int pv_topn_x_names(pv_ctx *c, const uint8_t *const *cands, const size_t *sizes, uint32_t n, uint8_t **blob, size_t *bytes)
{
    *blob = nullptr;
    *bytes = 0;
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    std::vector<XCand> want;
    for (uint32_t q = 0; q < n; q++) {
        std::vector<XCand> v;
        if (!x_parse_cands(cands[q], sizes[q], v)) return c->fail(PV_EINVAL, "malformed candidate blob %u", q);
        for (auto &x : v)
            if (!x.named) want.push_back(x);
    }
    std::vector<uint8_t> o;
    // each wanted key against every live table of its set's part (a rank may hold it in any period)
    {
        std::vector<XCand> w2;
        for (auto &x : want) {
            const int part = (int)(x.tb >> 16);
            for (uint32_t s : (part == PART_DNS ? c->dns.slots : c->net.slots)) {
                XCand y = x;
                y.tb = s + (part == PART_DNS ? PV_SLOTS : 0);
                y.name = std::to_string(x.tb); // (the set id, for the answer)
                w2.push_back(y);
            }
        }
        want.swap(w2);
    }
    if (!want.empty()) {
        std::vector<uint64_t> keys;
        std::vector<uint32_t> tbs;
        for (auto &x : want) { keys.push_back(x.key); tbs.push_back(x.tb); }
        PvParams P;
        if (int rc = x_params(c, P)) return rc;
        uint64_t *d_k = nullptr;
        uint32_t *d_t = nullptr, *d_a = nullptr;
        hipError_t e;
        std::vector<uint32_t> aux(want.size());
        if (!hip_ok(e = hipMalloc(&d_k, keys.size() * 8)) || !hip_ok(e = hipMalloc(&d_t, keys.size() * 4)) ||
            !hip_ok(e = hipMalloc(&d_a, keys.size() * 4))) {
            hipFree(d_k); hipFree(d_t); hipFree(d_a);
            return c->hipfail(e, "name lookup");
        }
        bool ok = hip_ok(e = hipMemcpy(d_k, keys.data(), keys.size() * 8, hipMemcpyHostToDevice)) &&
                  hip_ok(e = hipMemcpy(d_t, tbs.data(), tbs.size() * 4, hipMemcpyHostToDevice));
        if (ok) {
            hipLaunchKernelGGL(pv_topn_xlookup, dim3((uint32_t)((keys.size() + 255) / 256)), dim3(256), 0, c->stream,
                               (const PvParams *)c->d_xp, (const uint64_t *)d_k, (const uint32_t *)d_t, (uint32_t)keys.size(), d_a);
            ok = hip_ok(e = hipGetLastError()) && hip_ok(e = hipStreamSynchronize(c->stream)) &&
                 hip_ok(e = hipMemcpy(aux.data(), d_a, aux.size() * 4, hipMemcpyDeviceToHost));
        }
        hipFree(d_k); hipFree(d_t); hipFree(d_a);
        if (!ok) return c->hipfail(e, "name lookup");
        std::vector<uint32_t> gtb, gaux;
        std::vector<uint64_t> gkey;
        for (size_t i = 0; i < want.size(); i++) { gtb.push_back(want[i].tb); gaux.push_back(aux[i]); gkey.push_back(want[i].key); }
        std::vector<std::string> txt;
        std::vector<bool> okv;
        if (int rc = x_read_names(c, gtb, gaux, gkey, txt, okv)) return rc;
        std::set<std::pair<uint32_t, uint64_t>> done;
        for (size_t i = 0; i < want.size(); i++) {
            const uint32_t set = (uint32_t)std::stoul(want[i].name);
            if (done.count({set, want[i].key}) || !okv[i]) continue;
            done.insert({set, want[i].key});
            put_u32(o, set);
            put_u64(o, want[i].key);
            put_name(o, &txt[i]);
        }
    }
    *blob = (uint8_t *)malloc(std::max<size_t>(o.size(), 1));
    if (!*blob) return c->fail(PV_ECAPACITY, "name answers");
    memcpy(*blob, o.data(), o.size());
    *bytes = o.size();
    return 0;
}

int pv_topn_x_view(pv_ctx *c, const uint8_t *const *cands, const size_t *csizes, const uint8_t *const *names,
                   const size_t *nsizes, uint32_t n)
{
    mark_merged(c, "pv_topn_x_view");
    std::lock_guard<std::mutex> g(c->mu);
    std::map<std::pair<uint32_t, uint64_t>, std::string> known;
    for (uint32_t q = 0; q < n; q++) {
        const uint8_t *b = names[q];
        size_t p = 0, m = nsizes[q];
        while (p + 14 <= m) {
            uint32_t tb; uint64_t key; uint16_t l;
            memcpy(&tb, b + p, 4); memcpy(&key, b + p + 4, 8); memcpy(&l, b + p + 12, 2);
            if (l == 0xffff || p + 14 + l > m) return c->fail(PV_EINVAL, "malformed name blob %u", q);
            known[{tb, key}].assign((const char *)b + p + 14, l);
            p += 14 + l;
        }
    }
    c->x_view.clear();
    for (uint32_t q = 0; q < n; q++) {
        std::vector<XCand> v;
        if (!x_parse_cands(cands[q], csizes[q], v)) return c->fail(PV_EINVAL, "malformed candidate blob %u", q);
        for (auto &x : v) {
            std::string nm = x.name;
            if (!x.named) {
                auto it = known.find({x.tb, x.key});
                if (it != known.end()) nm = it->second;
            }
            c->x_view[x.tb][x.key] = {x.est, nm};
        }
    }
    c->x_view_on = true;
    return 0;
}

// ---- quantile inputs across shards without shipping the values: exact radix selection whose
// per-pass group histograms (256 bins, one byte of the value) are summed over the ranks by a
// caller-supplied all-reduce (pv_values_x_select) or RCCL (pv_comm_values_select). Per live DNS
// slot and value kind: the count, p50/p90/p95/p99 and the maximum (the KLL inclusive rank rule
// of Quantile, src/Metrics.h:334-481, on the union of the shards' values: what one stream
// gives) and, for the time kinds, the count at or below each histogram point (Histogram,
// src/Metrics.h:189-327). The merged view then holds a stand-in value list per slot and kind
// with those counts, that maximum and those quantiles.
namespace {
int x_allreduce(pv_ctx *c, pv_allreduce_fn ar, void *user, std::vector<uint64_t> &buf, int op)
{
    if (buf.empty()) return 0;
    if (ar) return ar(buf.data(), buf.size(), op, user) ? c->fail(PV_EINVAL, "all-reduce callback failed") : 0;
    // RCCL on the context's communicator
    hipError_t e;
    uint64_t *d = nullptr;
    if (!hip_ok(e = hipMalloc(&d, buf.size() * 8))) return c->hipfail(e, "selection all-reduce");
    ncclResult_t r = ncclSuccess;
    const bool ok = hip_ok(e = hipMemcpyAsync(d, buf.data(), buf.size() * 8, hipMemcpyHostToDevice, c->stream)) &&
                    (r = ncclAllReduce(d, d, buf.size(), ncclUint64, op ? ncclMax : ncclSum, c->comm, c->stream)) == ncclSuccess &&
                    hip_ok(e = hipMemcpyAsync(buf.data(), d, buf.size() * 8, hipMemcpyDeviceToHost, c->stream)) &&
                    hip_ok(e = hipStreamSynchronize(c->stream));
    hipFree(d);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllReduce: %s", ncclGetErrorString(r));
    if (!ok) return c->hipfail(e, "selection all-reduce");
    return 0;
}
// rank of fraction p among n values (quantiles(): ceil(p n) - 1, clamped); p > 1: the maximum
uint64_t x_rank_of(double p, uint64_t n)
{
    if (p > 1.0) return n ? n - 1 : 0;
    const uint64_t w = (uint64_t)std::ceil(p * (double)n);
    uint64_t idx = w == 0 ? 0 : w - 1;
    return n && idx >= n ? n - 1 : idx;
}
// Exact distributed selection. gparts[g]: this rank's values of group g, as sorted parts (a
// value lies in one part); fr[g]: the fractions wanted. out[g][k]: the value at each fraction's
// rank over every rank's values (0 when the group is empty everywhere); n[g]: the group's count
// over every rank. Eight passes, one byte each from the top: per target the 256-bin histogram of
// the values whose higher bytes equal the target's prefix so far, all-reduced (one call per
// pass), then the bin holding the target's rank. The bins are counted by binary searches over the
// sorted parts (257 bin edges per part), so a pass costs O(targets x parts x 256 log n), not a
// scan of every value per target.
using XParts = std::vector<const std::vector<uint64_t> *>;
int x_select(pv_ctx *c, pv_allreduce_fn ar, void *user, const std::vector<XParts> &gparts,
             const std::vector<std::vector<double>> &fr, std::vector<uint64_t> &n, std::vector<std::vector<uint64_t>> &out)
{
    const size_t G = gparts.size();
    struct Tg { uint32_t g; double p; uint64_t rank, prefix; };
    std::vector<Tg> T;
    for (uint32_t g = 0; g < G; g++)
        for (double p : fr[g]) T.push_back(Tg{g, p, 0, 0});
    n.assign(G, 0);
    out.assign(G, {});
    // values <= x in a group's parts
    auto count_le = [&](const XParts &ps, uint64_t x) {
        uint64_t k = 0;
        for (const std::vector<uint64_t> *v : ps) k += (uint64_t)(std::upper_bound(v->begin(), v->end(), x) - v->begin());
        return k;
    };
    std::vector<uint64_t> h;
    for (int pass = 0; pass < 8; pass++) {
        const uint32_t shift = 56 - 8 * pass;
        h.assign(T.size() * 256, 0);
        std::map<std::pair<uint32_t, uint64_t>, size_t> done; // (group, range) -> target that counted it
        for (size_t t = 0; t < T.size(); t++) {
            const XParts &ps = gparts[T[t].g];
            // the target's range: its prefix above this byte, every value of the lower bytes
            const uint64_t base = pass == 0 ? 0ull : T[t].prefix & (~0ull << (shift + 8));
            auto it = done.find({T[t].g, base});
            if (it != done.end()) {
                std::copy(h.begin() + it->second * 256, h.begin() + it->second * 256 + 256, h.begin() + t * 256);
                continue;
            }
            done[{T[t].g, base}] = t;
            uint64_t below = base ? count_le(ps, base - 1) : 0;
            for (uint32_t bn = 0; bn < 256; bn++) {
                const uint64_t top = base + ((uint64_t)bn << shift) + ((1ull << shift) - 1);
                const uint64_t le = count_le(ps, top);
                h[t * 256 + bn] = le - below;
                below = le;
            }
        }
        if (int rc = x_allreduce(c, ar, user, h, 0)) return rc;
        for (size_t t = 0; t < T.size(); t++) {
            const uint64_t *hh = &h[t * 256];
            if (pass == 0) {
                uint64_t tot = 0;
                for (int b = 0; b < 256; b++) tot += hh[b];
                n[T[t].g] = tot;
                T[t].rank = x_rank_of(T[t].p, tot);
            }
            if (!n[T[t].g]) continue;
            uint64_t cum = 0;
            int b = 0;
            while (b < 255 && cum + hh[b] <= T[t].rank) cum += hh[b++];
            T[t].rank -= cum;
            T[t].prefix |= (uint64_t)b << shift;
        }
    }
    for (auto &t : T) out[t.g].push_back(n[t.g] ? t.prefix : 0);
    return 0;
}
const uint32_t X_KINDS[9] = {XV_FROM_US, XV_TO_US, XV_RATIO, XV2_TIME, XV2_TIME + 1, XV2_TIME + 2, XV2_RATIO, XV2_RATIO + 1, XV2_RATIO + 2};
bool x_time_kind(uint32_t k) { return k == XV_FROM_US || k == XV_TO_US || (k >= XV2_TIME && k < XV2_TIME + 3); }

int values_select(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = sync_xvals(c)) return rc;
    // groups: (slot set, kind), the sets a window read can ask for: each live DNS slot alone
    // (window_json of one period) and each run of the most recent slots (merged windows)
    std::vector<uint32_t> sets;
    for (uint32_t s : c->dns.slots) sets.push_back(1u << s);
    {
        uint32_t m = 0;
        for (size_t i = 0; i < c->dns.slots.size(); i++) {
            m |= 1u << c->dns.slots[i];
            if (i) sets.push_back(m);
        }
    }
    const size_t G = sets.size() * 9;
    std::vector<std::vector<double>> fr(G, std::vector<double>{0.50, 0.90, 0.95, 0.99, 2.0});
    // the values by (live slot, kind), each sorted once; a group (slot set, kind) is the parts of
    // its slots
    std::map<uint32_t, uint32_t> sg_idx; // live slot | gen << 8 -> its index among the live slots
    for (size_t i = 0; i < c->dns.slots.size(); i++) sg_idx[c->dns.slots[i] | (c->gen[c->dns.slots[i]] << 8)] = (uint32_t)i;
    const size_t NS = c->dns.slots.size();
    std::vector<std::vector<uint64_t>> part(NS * 9);
    for (const PvXValue &v : c->xvals_host) {
        auto it = sg_idx.find(v.slot);
        if (it == sg_idx.end()) continue;
        int k = 0;
        while (k < 9 && v.kind != X_KINDS[k]) k++;
        if (k == 9) continue;
        part[(size_t)it->second * 9 + k].push_back(v.bits);
    }
    for (auto &v : part) std::sort(v.begin(), v.end());
    std::vector<XParts> groups(G);
    for (size_t i = 0; i < sets.size(); i++)
        for (size_t si = 0; si < NS; si++)
            if (sets[i] & (1u << c->dns.slots[si]))
                for (int k = 0; k < 9; k++) groups[i * 9 + k].push_back(&part[si * 9 + k]);
    std::vector<uint64_t> n;
    std::vector<std::vector<uint64_t>> q;
    if (int rc = x_select(c, ar, user, groups, fr, n, q)) return rc;
    // counts at or below each histogram point, time kinds
    const std::vector<uint64_t> &pts = hist_points();
    std::vector<uint64_t> cdf(G * pts.size(), 0);
    for (size_t gi = 0; gi < G; gi++) {
        if (!x_time_kind(X_KINDS[gi % 9])) continue;
        for (size_t k = 0; k < pts.size(); k++)
            for (const std::vector<uint64_t> *v : groups[gi])
                cdf[gi * pts.size() + k] += (uint64_t)(std::upper_bound(v->begin(), v->end(), pts[k]) - v->begin());
    }
    if (int rc = x_allreduce(c, ar, user, cdf, 0)) return rc;
    c->xq.clear();
    for (size_t gi = 0; gi < G; gi++) {
        if (!n[gi]) continue;
        XQuant &x = c->xq[{sets[gi / 9], X_KINDS[gi % 9]}];
        x.n = n[gi];
        x.q.assign(q[gi].begin(), q[gi].begin() + 4);
        x.max = q[gi][4];
        if (x_time_kind(X_KINDS[gi % 9])) x.cdf.assign(cdf.begin() + gi * pts.size(), cdf.begin() + (gi + 1) * pts.size());
    }
    c->xq_on = true;
    return 0;
}
} // namespace

int pv_values_x_select(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    mark_merged(c, "pv_values_x_select");
    if (!ar) return c->fail(PV_EINVAL, "no all-reduce callback");
    return values_select(c, ar, user);
}

int pv_comm_values_select(pv_ctx *c)
{
    mark_merged(c, "pv_comm_values_select");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    return values_select(c, nullptr, nullptr);
}

// The device regions of both live windows a multi-GPU reduce combines: each Net slot's
// net part and each DNS slot's dns part of the SUM (all-reduce SUM) and MIN (all-reduce MIN)
// words. The caller writes them, so they stop being clean.
int pv_window_regions(pv_ctx *c, pv_region *r, uint32_t max, uint32_t *n)
{
    mark_merged(c, "pv_window_regions");
    std::lock_guard<std::mutex> g(c->mu);
    flush_fills(c);
    std::vector<pv_region> v;
    // the parts of each slot the attached handler versions use (the others stay zero)
    auto sum = [&](uint32_t s, size_t a, size_t b) { v.push_back(pv_region{c->d_sum + (size_t)s * PV_SUM_WORDS + a, b - a, PV_REDUCE_SUM, 0}); };
    auto cpc = [&](uint32_t s, size_t k0, size_t k1) {
        v.push_back(pv_region{c->d_cpc + (size_t)s * PV_MIN_WORDS + k0 * PV_CPC_COUPONS, (k1 - k0) * PV_CPC_COUPONS,
                              PV_REDUCE_MIN, 0});
    };
    for (uint32_t s : c->net.slots) {
        sum(s, 0, PV_OFF_NET2);
        cpc(s, CPC_SRC, CPC_V2);
        if (c->net2_groups) { sum(s, PV_OFF_NET2, PV_SUM_NET_WORDS); cpc(s, CPC_V2, CPC_QNAME); }
        c->net.clean[s] = false;
    }
    for (uint32_t s : c->dns.slots) {
        if (c->dns2_groups) {
            sum(s, PV_OFF_DNS, PV_OFF_DNS + PV_DNS_CTRS);
            sum(s, PV_OFF_DNS2, PV_SUM_WORDS);
            cpc(s, CPC_QNAME2, CPC_QNAME2 + 3);
        } else {
            sum(s, PV_OFF_DNS, PV_OFF_DNS2);
            cpc(s, CPC_QNAME, CPC_QNAME + 1);
        }
        c->dns.clean[s] = false;
    }
    *n = (uint32_t)v.size();
    for (uint32_t i = 0; i < v.size() && i < max; i++) r[i] = v[i];
    return 0;
}

int pv_comm_unique_id(uint8_t id[PV_COMM_ID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) == PV_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PV_EHIP;
    memcpy(id, &u, sizeof u);
    return 0;
}

int pv_comm_init(pv_ctx *c, const uint8_t id[PV_COMM_ID_BYTES], int nranks, int rank)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (c->comm) return c->fail(PV_EINVAL, "communicator already initialised");
    if (nranks < 1 || rank < 0 || rank >= nranks) return c->fail(PV_EINVAL, "rank %d of %d", rank, nranks);
    hipSetDevice(c->device);
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        return c->fail(PV_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    c->comm_ranks = nranks;
    c->comm_rank = rank;
    return 0;
}

int pv_comm_allreduce_window(pv_ctx *c)
{
    mark_merged(c, "pv_comm_allreduce_window");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    std::vector<pv_region> v(8 * PV_SLOTS);
    uint32_t n = 0;
    if (int rc = pv_window_regions(c, v.data(), (uint32_t)v.size(), &n)) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    flush_fills(c);
    ncclResult_t r = ncclGroupStart();
    for (uint32_t i = 0; i < n && r == ncclSuccess; i++)
        r = ncclAllReduce(v[i].ptr, v[i].ptr, v[i].words, v[i].op == PV_REDUCE_SUM ? ncclUint64 : ncclInt64,
                          v[i].op == PV_REDUCE_SUM ? ncclSum : ncclMin, c->comm, c->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) return c->fail(PV_EHIP, "ncclAllReduce: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    hipError_t e;
    if (!hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "window all-reduce");
    return 0;
}

// all-gather of one equal-sized host block per rank (the caller holds c->mu)
int comm_allgather_locked(pv_ctx *c, const void *buf, size_t bytes, std::vector<uint8_t> &out)
{
    const int R = c->comm_ranks;
    out.assign((size_t)R * bytes, 0);
    if (!bytes) return 0;
    hipError_t e;
    uint8_t *d = nullptr;
    if (!hip_ok(e = hipMalloc(&d, bytes * (R + 1)))) return c->hipfail(e, "all-gather buffers");
    ncclResult_t r = ncclSuccess;
    bool ok = hip_ok(e = hipMemcpyAsync(d + bytes * R, buf, bytes, hipMemcpyHostToDevice, c->stream)) &&
              (r = ncclAllGather(d + bytes * R, d, bytes, ncclUint8, c->comm, c->stream)) == ncclSuccess &&
              hip_ok(e = hipMemcpyAsync(out.data(), d, bytes * R, hipMemcpyDeviceToHost, c->stream)) &&
              hip_ok(e = hipStreamSynchronize(c->stream));
    hipFree(d);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    if (!ok) return c->hipfail(e, "all-gather");
    return 0;
}

int pv_comm_allgather(pv_ctx *c, const void *buf, size_t bytes, uint8_t **out, uint64_t *sizes)
{
    *out = nullptr;
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    const int R = c->comm_ranks;
    hipError_t e;
    uint64_t *d_sz = nullptr;
    uint8_t *d_in = nullptr, *d_all = nullptr;
    struct Free {
        void *a, *b, *c;
        ~Free() { for (void *p : {a, b, c}) if (p) hipFree(p); }
    } fr{nullptr, nullptr, nullptr};
    if (!hip_ok(e = hipMalloc(&d_sz, (size_t)R * 16))) return c->hipfail(e, "all-gather sizes");
    fr.a = d_sz;
    const uint64_t mine = bytes;
    if (!hip_ok(e = hipMemcpyAsync(d_sz + R, &mine, 8, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "all-gather sizes");
    ncclResult_t r = ncclAllGather(d_sz + R, d_sz, 1, ncclUint64, c->comm, c->stream);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    if (!hip_ok(e = hipMemcpyAsync(sizes, d_sz, (size_t)R * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "all-gather sizes");
    uint64_t mx = 0, tot = 0;
    for (int k = 0; k < R; k++) { mx = std::max(mx, sizes[k]); tot += sizes[k]; }
    const size_t chunk = (size_t)std::max<uint64_t>(mx, 1);
    if (!hip_ok(e = hipMalloc(&d_in, chunk)) || !hip_ok(e = hipMalloc(&d_all, chunk * R))) return c->hipfail(e, "all-gather buffers");
    fr.b = d_in;
    fr.c = d_all;
    if (bytes && !hip_ok(e = hipMemcpyAsync(d_in, buf, bytes, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "all-gather upload");
    r = ncclAllGather(d_in, d_all, chunk, ncclUint8, c->comm, c->stream);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    std::vector<uint8_t> all(chunk * R);
    if (!hip_ok(e = hipMemcpyAsync(all.data(), d_all, all.size(), hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "all-gather download");
    uint8_t *o = (uint8_t *)malloc(std::max<uint64_t>(tot, 1));
    if (!o) return c->fail(PV_ECAPACITY, "all-gather result");
    uint64_t at = 0;
    for (int k = 0; k < R; k++) { memcpy(o + at, all.data() + (size_t)k * chunk, sizes[k]); at += sizes[k]; }
    *out = o;
    return 0;
}

int pv_comm_destroy(pv_ctx *c)
{
    if (!c->comm) return 0;
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
    return 0;
}

int pv_set_kernel_timing(pv_ctx *c, uint32_t every)
{
    c->timing_every = every;
    c->timing_ctr = 0;
    return 0;
}

int pv_kernel_timing(pv_ctx *c, double *total_ms, uint64_t *launches, int reset)
{
    *total_ms = c->kernel_ms;
    *launches = c->kernel_launches;
    if (reset) { c->kernel_ms = 0; c->kernel_launches = 0; }
    return 0;
}

// ---- multi-GPU shard edges: DNS transactions across contiguous shards.
// Each rank exports its shard-edge stubs: the queries still open at the end of its
// stream (latest per (flow, txid)), its orphan responses (first event of their key in
// its stream) and its DNS period shifts. Every rank then replays the ranks before it:
// the open queries of shard j that shards j+1 .. r-1 neither answered nor purged reach
// shard r, where they pair with r's orphan responses (TransactionManager::
// maybe_end_transaction, libs/visor_transaction/TransactionManager.h:51-106) or time out
// at r's period shifts (DnsStreamHandler.h:252-267). Each rank counts only what happens
// in its own shard, into its own buckets, before the bucket all-reduce.
namespace {
struct EdgeHdr {
    uint32_t magic, n_open, n_orph, n_shift;
};
const uint32_t EDGE_MAGIC = 0x31455650u; // "PVE1"
struct EdgeView {
    std::vector<PvXEvent> open, orph;
    std::vector<std::pair<int64_t, uint32_t>> shifts;
};
bool edge_parse(const uint8_t *b, size_t n, EdgeView &v)
{
    EdgeHdr h;
    if (n < sizeof h) return false;
    memcpy(&h, b, sizeof h);
    const size_t need = sizeof h + ((size_t)h.n_open + h.n_orph) * sizeof(PvXEvent) + (size_t)h.n_shift * 12;
    if (h.magic != EDGE_MAGIC || n != need) return false;
    const uint8_t *p = b + sizeof h;
    v.open.resize(h.n_open);
    v.orph.resize(h.n_orph);
    if (h.n_open) memcpy(v.open.data(), p, h.n_open * sizeof(PvXEvent));
    p += h.n_open * sizeof(PvXEvent);
    if (h.n_orph) memcpy(v.orph.data(), p, h.n_orph * sizeof(PvXEvent));
    p += h.n_orph * sizeof(PvXEvent);
    v.shifts.resize(h.n_shift);
    for (uint32_t i = 0; i < h.n_shift; i++) {
        memcpy(&v.shifts[i].first, p + 12 * i, 8);
        memcpy(&v.shifts[i].second, p + 12 * i + 8, 4);
    }
    return true;
}
// first shift of `sh` at or after ttl + sec (the purge of a query started at sec), or -1
int purge_shift(const std::vector<std::pair<int64_t, uint32_t>> &sh, uint32_t ttl_s, int64_t sec)
{
    for (size_t i = 0; i < sh.size(); i++)
        if (sh[i].first >= (int64_t)ttl_s + sec) return (int)i;
    return -1;
}
int add_dns_words(pv_ctx *c, uint32_t slot, const uint64_t add[4])
{
    static const int w[4] = {DC_XTOTAL, DC_XOUT, DC_XIN, DC_XTIMEOUT};
    c->dns.clean[slot] = false;
    for (int k = 0; k < 4; k++) {
        if (!add[k]) continue;
        uint64_t *dp = c->d_sum + (size_t)slot * PV_SUM_WORDS + PV_OFF_DNS + w[k];
        uint64_t v = 0;
        hipError_t e;
        if (!hip_ok(e = hipMemcpy(&v, dp, 8, hipMemcpyDeviceToHost))) return c->hipfail(e, "edge counters");
        v += add[k];
        if (!hip_ok(e = hipMemcpy(dp, &v, 8, hipMemcpyHostToDevice))) return c->hipfail(e, "edge counters");
    }
    return 0;
}
bool in_dns_window(pv_ctx *c, uint32_t slot)
{
    return std::find(c->dns.slots.begin(), c->dns.slots.end(), slot) != c->dns.slots.end();
}
// the carried list on the host: each open query event (gathered from the event store by its
// index) with its sort key
int read_carried(pv_ctx *c, std::vector<PvXEvent> &pend, std::vector<uint64_t> &pk, std::vector<uint64_t> *ecs = nullptr)
{
    pend.clear();
    pk.assign(c->n_pend, 0);
    if (ecs) ecs->assign(c->n_pend, 0);
    if (!c->n_pend) return 0;
    std::vector<uint32_t> pv(c->n_pend);
    std::vector<PvXEvent> store(c->pend_hi);
    std::vector<uint64_t> estore(ecs && c->d_pecs[c->pend_cur] ? c->pend_hi : 0);
    hipError_t e;
    if (!hip_ok(e = hipMemcpy(pk.data(), c->d_pkeys[c->pend_cur], c->n_pend * 8, hipMemcpyDeviceToHost)) ||
        !hip_ok(e = hipMemcpy(pv.data(), c->d_pvals[c->pend_cur], c->n_pend * 4, hipMemcpyDeviceToHost)) ||
        !hip_ok(e = hipMemcpy(store.data(), c->d_pend[c->pend_cur], c->pend_hi * sizeof(PvXEvent), hipMemcpyDeviceToHost)) ||
        (!estore.empty() && !hip_ok(e = hipMemcpy(estore.data(), c->d_pecs[c->pend_cur], c->pend_hi * 8, hipMemcpyDeviceToHost))))
        return c->hipfail(e, "open queries");
    pend.resize(c->n_pend);
    for (size_t i = 0; i < pv.size(); i++) {
        if (pv[i] >= c->pend_hi) return c->fail(PV_EINVAL, "carried query %zu indexes past the event store", i);
        pend[i] = store[pv[i]];
        if (!estore.empty()) (*ecs)[i] = estore[pv[i]];
    }
    return 0;
}
// one SUM word of a slot += delta (host read-modify-write: the few counters an edge merge moves)
int add_sum_word(pv_ctx *c, uint32_t slot, uint32_t word, int64_t delta)
{
    if (!delta) return 0;
    c->dns.clean[slot] = false;
    uint64_t *dp = c->d_sum + (size_t)slot * PV_SUM_WORDS + word;
    uint64_t v = 0;
    hipError_t e;
    if (!hip_ok(e = hipMemcpy(&v, dp, 8, hipMemcpyDeviceToHost))) return c->hipfail(e, "edge counters");
    v += (uint64_t)delta;
    if (!hip_ok(e = hipMemcpy(dp, &v, 8, hipMemcpyHostToDevice))) return c->hipfail(e, "edge counters");
    return 0;
}

// pv_edge_carry for DNS v2 (one TransactionManager per transaction direction, the direction in
// the key; dns/v2/DnsStreamHandler.cpp:1100-1145, the manager's purge at its shifts .h:440-453):
// an open query meets the first event of its key in this shard as resolve_one2 would have met it
// in one stream. A response there, which this shard counted as an orphan, pairs instead: the
// orphan count is taken back and the transaction accounted on the response (pv_xact_edge2), or
// counted filtered / timed out. Purges are time-outs of the purging shift's bucket. The edge
// pairs' times feed the stream's thresholds (slow_xv) and their slow candidates (scands).
// Buffers: n x (PvXEvent [+ u64 ECS address with top_ecs]).
// The first stub (this shard's first event) of each incoming open query's key: a map over the
// incoming keys (usually few) and one scan of the stubs in first-occurrence order, instead of a map
// over every stub of the shard (millions in a shard the edge horizon covers whole: the map's build
// was most of each rank's turn in the edge chain).
static void edge_first_stubs(const pv_ctx *c, const uint8_t *in, size_t n, size_t esz, std::unordered_map<uint64_t, size_t> &first)
{
    first.reserve(n * 2);
    for (size_t k = 0; k < n; k++) {
        uint64_t key;
        memcpy(&key, in + k * esz + offsetof(PvXEvent, key), 8);
        first.emplace(key, SIZE_MAX);
    }
    if (first.empty()) return;
    size_t left = first.size();
    for (size_t i = 0; i < c->stubs.size() && left; i++) {
        auto it = first.find(c->stubs[i].e.key);
        if (it != first.end() && it->second == SIZE_MAX) { it->second = i; left--; }
    }
    for (auto it = first.begin(); it != first.end();) it = it->second == SIZE_MAX ? first.erase(it) : std::next(it);
}

int edge_carry2(pv_ctx *c, const uint8_t *in, size_t in_bytes, uint8_t **out, size_t *out_bytes)
{
    const bool ecs = c->d_pecs[0] != nullptr;
    const size_t esz = sizeof(PvXEvent) + (ecs ? 8 : 0);
    if (in_bytes % esz) return c->fail(PV_EINVAL, "malformed open-query buffer");
    std::unordered_map<uint64_t, size_t> first;
    edge_first_stubs(c, in, in_bytes / esz, esz, first);
    const uint64_t live = c->dns.ordinal;
    auto in_win = [&](uint64_t ord) { return ord <= live && ord + c->dns.slots.size() > live; };
    auto slot_of = [&](uint64_t ord) { return c->dns.slots[live - ord]; };
    const uint32_t g = c->dns2_groups;
    std::map<std::pair<uint32_t, uint32_t>, int64_t> add; // (slot, SUM word) -> delta
    std::vector<PvXEvent> keep;
    std::vector<uint64_t> keep_ecs;
    std::vector<PvEdgePair> pairs;
    std::vector<size_t> pair_stub;
    const size_t nin = in_bytes / esz;
    for (size_t k = 0; k < nin; k++) {
        PvXEvent qe;
        uint64_t qaddr = 0;
        memcpy(&qe, in + k * esz, sizeof qe);
        if (ecs) memcpy(&qaddr, in + k * esz + sizeof qe, 8);
        const uint32_t xd = (uint32_t)((qe.key >> 48) & 3) - 1;
        if (xd >= 3) return c->fail(PV_EINVAL, "open query %zu has no DNS v2 transaction direction", k);
        auto d2 = [&](uint32_t slot, uint32_t ctr, int64_t v) { add[{slot, PV_OFF_DNS2 + xd * PV_DNS2_CTRS + ctr}] += v; };
        int ps = -1;
        for (size_t i = 0; i < c->dns_shift_ord.size(); i++)
            if (c->dns_shift_ord[i].first >= (int64_t)c->ttl_s + qe.sec) { ps = (int)i; break; }
        auto purged = [&]() {
            const uint64_t o = c->dns_shift_ord[ps].second;
            if (in_win(o)) { d2(slot_of(o), D2_TIMEOUT, 1); d2(slot_of(o), D2_SEEN, 1); }
        };
        auto it = first.find(qe.key);
        if (it == first.end()) {
            if (ps >= 0) purged();
            else { keep.push_back(qe); keep_ecs.push_back(qaddr); }
            continue;
        }
        const pv_ctx::EdgeStub &st = c->stubs[it->second];
        if (ps >= 0 && st.ord >= c->dns_shift_ord[ps].second) { purged(); continue; } // purged before its key's next event
        if (!st.e.qr) continue;                                                          // overwritten by a new query
        const PvXEvent &r = st.e;
        const bool win = in_win(st.ord), kept = (r.period & 0x80) && win;
        const uint32_t slot = win ? slot_of(st.ord) : 0;
        const bool rf = r.pad & 4, qf = qe.pad & 4, rdeep = !(r.pad & 32);
        int64_t dsec = r.sec > qe.sec ? r.sec - qe.sec : qe.sec - r.sec;
        int64_t dnsec = (int64_t)r.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        const bool timed_out = dsec > (int64_t)c->ttl_s || (dsec == (int64_t)c->ttl_s && ((double)dnsec / 1.0e6) >= (double)c->ttl_ms);
        if (kept && !rf) d2(slot, D2_ORPHAN, -1); // this shard counted it NotExist; it is Valid / TimedOut
        auto filtered = [&]() { if (kept && (g & PV_D2G_COUNTERS)) add[{slot, PV_OFF_DNS + DC_FILTERED}] += 1; };
        if (rf) { if (!timed_out && !qf) filtered(); continue; }
        if (qf) { filtered(); continue; }
        if (timed_out) { if (kept) d2(slot, D2_TIMEOUT, 1); continue; }
        const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        const PvXValue tv{us, 0, (uint32_t)XV2_TIME + xd};
        if (!(r.period & 0x80)) { // a period outside the window then: its time feeds the next p90 only
            if (g & PV_D2G_XACT_TIMES) c->slow_xv.push_back({st.ord, tv});
            continue;
        }
        if ((g & PV_D2G_XACT_TIMES) && rdeep) c->slow_xv.push_back({st.ord, tv});
        if (!win) continue; // its bucket has left the window since
        if ((g & PV_D2G_XACT_TIMES) && rdeep && st.cand >= 0) {
            pv_ctx::SlowCand sc = c->sorph[(size_t)st.cand];
            sc.us = us;
            sc.dir = (uint8_t)(4 + xd);
            c->scands.push_back(sc);
        }
        if (st.cand < 0) return c->fail(PV_EINVAL, "shard-edge response without its record");
        pairs.push_back(PvEdgePair{qe, r, qaddr, st.order, us});
        pair_stub.push_back(it->second);
    }
    for (auto &kv : add)
        if (int rc = add_sum_word(c, kv.first.first, kv.first.second, kv.second)) return rc;
    // the edge pairs on the device, by groups of at most PV_MAX_SHIFTS + 1 periods (the edge
    // run's period table)
    std::vector<uint64_t> ords;
    for (size_t i : pair_stub) ords.push_back(c->stubs[i].ord);
    std::sort(ords.begin(), ords.end());
    ords.erase(std::unique(ords.begin(), ords.end()), ords.end());
    hipError_t e;
    for (size_t g0 = 0; g0 < ords.size(); g0 += PV_MAX_SHIFTS + 1) {
        const size_t g1 = std::min(ords.size(), g0 + PV_MAX_SHIFTS + 1);
        std::vector<uint8_t> blob[2];
        std::vector<uint32_t> offs[2];
        std::vector<PvEdgePair> run;
        for (size_t i = 0; i < pairs.size(); i++) {
            const pv_ctx::EdgeStub &st = c->stubs[pair_stub[i]];
            auto itp = std::find(ords.begin() + g0, ords.begin() + g1, st.ord);
            if (itp == ords.begin() + g1) continue;
            const pv_ctx::SlowCand &sc = c->sorph[(size_t)st.cand];
            const uint8_t *rec = c->sstore.data() + sc.off;
            uint32_t cap;
            memcpy(&cap, rec + 8, 4);
            const uint32_t sz = (16 + cap + 3) & ~3u;
            offs[sc.tcp].push_back((uint32_t)blob[sc.tcp].size());
            blob[sc.tcp].insert(blob[sc.tcp].end(), rec, rec + sz);
            PvEdgePair pp = pairs[i];
            pp.r.idx = (uint32_t)(offs[sc.tcp].size() - 1) | (sc.tcp ? PV_TCP_IDX : 0u);
            pp.r.period = (uint8_t)(itp - (ords.begin() + g0));
            run.push_back(pp);
        }
        if (run.empty()) continue;
        for (int k = 0; k < 2; k++) blob[k].resize(blob[k].size() + PV_RECS_PAD, 0);
        void *d[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        struct Free { void **p; ~Free() { for (int i = 0; i < 7; i++) if (p[i]) hipFree(p[i]); } } fr{d};
        for (int k = 0; k < 2; k++) {
            if (!hip_ok(e = hipMalloc(&d[2 * k], blob[k].size())) || !hip_ok(e = hipMalloc(&d[2 * k + 1], (offs[k].size() + 1) * 4)) ||
                !hip_ok(e = hipMalloc(&d[4 + k], offs[k].size() + 1)) ||
                !hip_ok(e = hipMemcpy(d[2 * k], blob[k].data(), blob[k].size(), hipMemcpyHostToDevice)) ||
                (!offs[k].empty() && !hip_ok(e = hipMemcpy(d[2 * k + 1], offs[k].data(), offs[k].size() * 4, hipMemcpyHostToDevice))))
                return c->hipfail(e, "edge pairs");
        }
        if (!hip_ok(e = hipMalloc(&d[6], run.size() * sizeof(PvEdgePair))) ||
            !hip_ok(e = hipMemcpy(d[6], run.data(), run.size() * sizeof(PvEdgePair), hipMemcpyHostToDevice)))
            return c->hipfail(e, "edge pairs");
        PvParams P;
        params_common(c, P, (const uint8_t *)d[0], (const uint32_t *)d[1], offs[0].size());
        P.sum = c->d_sum;
        P.cpc = c->d_cpc;
        P.tkeys = c->d_tkeys;
        P.tcnt = c->d_tcnt;
        P.taux = c->d_taux;
        P.tcap_log2 = c->tcap_log2;
        P.reg_log2 = c->reg_log2;
        P.arena = c->d_arena;
        P.arena_top = c->d_arena_top;
        P.arena_cap = c->arena_cap;
        P.tab_live = c->d_tab_live;
        P.flags = c->d_status + ST_FLAGS;
        P.sfx_of = (uint8_t *)d[4];
        P.n_dshift = (uint32_t)(g1 - g0 - 1);
        PvXactParams X;
        memset(&X, 0, sizeof X); // thresholds 0: the slow candidates are the host's (scands)
        for (size_t j = g0; j < g1; j++) {
            const uint32_t k = (uint32_t)(j - g0), slot = slot_of(ords[j]);
            P.dslot_of[k] = slot;
            X.slot_gen[k] = slot | (c->gen[slot] << 8);
            c->dns.clean[slot] = false;
        }
        X.P = P;
        X.vals = c->d_xvals;
        X.n_vals = c->d_nvals;
        X.vals_cap = (uint32_t)c->xv_cap;
        X.valid = c->d_valid;
        X.n_valid = c->d_nvals + 1;
        X.trecs = (const uint8_t *)d[2];
        X.toffs = (const uint32_t *)d[3];
        X.tsfx = (const uint8_t *)d[5];
        flush_fills(c);
        *c->h_xparams = X;
        if (!hip_ok(e = hipMemcpyAsync(c->d_xparams, c->h_xparams, sizeof X, hipMemcpyHostToDevice, c->stream)))
            return c->hipfail(e, "edge pairs");
        hipLaunchKernelGGL(pv_xact_edge2, dim3((uint32_t)((run.size() + 255) / 256)), dim3(256), 0, c->stream,
                           (const PvXactParams *)c->d_xparams, (const PvEdgePair *)d[6], (uint32_t)run.size(), (uint8_t *)d[4],
                           (uint8_t *)d[5]);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "pv_xact_edge2");
    }
    uint32_t flags = 0;
    if (!hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
    // this shard's own open queries (the carried list, latest event per key) with their ECS words
    if (c->n_pend) {
        std::vector<PvXEvent> pend;
        std::vector<uint64_t> pk, pe;
        if (int rc = read_carried(c, pend, pk, &pe)) return rc;
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(pend.size() * 2);
        for (size_t i = 0; i < pend.size(); i++) {
            auto it = last.find(pend[i].key);
            if (it == last.end() || (uint32_t)pk[i] >= (uint32_t)pk[it->second]) last[pend[i].key] = i;
        }
        for (auto &kv : last) { keep.push_back(pend[kv.second]); keep_ecs.push_back(pe[kv.second]); }
    }
    *out_bytes = keep.size() * esz;
    *out = (uint8_t *)malloc(*out_bytes ? *out_bytes : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "out of host memory");
    for (size_t i = 0; i < keep.size(); i++) {
        memcpy(*out + i * esz, &keep[i], sizeof(PvXEvent));
        if (ecs) memcpy(*out + i * esz + sizeof(PvXEvent), &keep_ecs[i], 8);
    }
    return 0;
}
} // namespace

int pv_edge_export(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    uint32_t nv[4];
    if (!hip_ok(e = hipMemcpy(nv, c->d_nvals, 16, hipMemcpyDeviceToHost))) return c->hipfail(e, "edge counts");
    if (nv[3] > c->orph_cap) return c->fail(PV_ECAPACITY, "%u shard-edge responses exceed the stub capacity", nv[3]);
    // open queries: the carried list, latest event per key (rank order in the sort keys)
    std::vector<PvXEvent> pend, open;
    std::vector<uint64_t> pk;
    if (int rc = read_carried(c, pend, pk)) return rc;
    if (c->n_pend) {
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(pend.size() * 2);
        for (size_t i = 0; i < pend.size(); i++) {
            auto it = last.find(pend[i].key);
            if (it == last.end() || (uint32_t)pk[i] >= (uint32_t)pk[it->second]) last[pend[i].key] = i;
        }
        open.reserve(last.size());
        for (auto &kv : last) open.push_back(pend[kv.second]);
    }
    std::vector<PvXEvent> orph(nv[3]);
    if (nv[3] && !hip_ok(e = hipMemcpy(orph.data(), c->d_orph, nv[3] * sizeof(PvXEvent), hipMemcpyDeviceToHost)))
        return c->hipfail(e, "edge responses");
    EdgeHdr h{EDGE_MAGIC, (uint32_t)open.size(), (uint32_t)orph.size(), (uint32_t)c->dns_shifts.size()};
    const size_t n = sizeof h + (open.size() + orph.size()) * sizeof(PvXEvent) + c->dns_shifts.size() * 12;
    uint8_t *o = (uint8_t *)malloc(n);
    if (!o) return c->fail(PV_ECAPACITY, "out of host memory");
    memcpy(o, &h, sizeof h);
    uint8_t *p = o + sizeof h;
    if (!open.empty()) memcpy(p, open.data(), open.size() * sizeof(PvXEvent));
    p += open.size() * sizeof(PvXEvent);
    if (!orph.empty()) memcpy(p, orph.data(), orph.size() * sizeof(PvXEvent));
    p += orph.size() * sizeof(PvXEvent);
    for (auto &sh : c->dns_shifts) {
        memcpy(p, &sh.first, 8);
        memcpy(p + 8, &sh.second, 4);
        p += 12;
    }
    *buf = o;
    *bytes = n;
    return 0;
}

int pv_edge_merge(pv_ctx *c, const uint8_t *const *bufs, const size_t *sizes, uint32_t nranks, uint32_t me)
{
    mark_merged(c, "pv_edge_merge");
    if (c->dns2_groups)
        return c->fail(PV_EUNSUPPORTED, "DNS v2 shard edges go rank by rank: pv_set_slow_defer, then pv_edge_carry");
    if (c->slow_defer) {
        // this rank's own transaction times end here (the edge pairs' follow)
        if (int rc = sync_xvals(c)) return rc;
        c->xv_local_end = c->xvals_host.size();
    }
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (me >= nranks) return c->fail(PV_EINVAL, "rank %u of %u", me, nranks);
    std::vector<EdgeView> v(nranks);
    for (uint32_t j = 0; j <= me; j++)
        if (!edge_parse(bufs[j], sizes[j], v[j])) return c->fail(PV_EINVAL, "malformed shard-edge buffer of rank %u", j);
    // queries open at the start of shard me, as the ranks before it leave them. A shift of shard j
    // purges every query with sec + ttl <= its second, so shard j purges the queries at or below
    // (its last shift - ttl): taken from a min-heap by second (entries a later query of the key or an
    // answer replaced are skipped by their sequence number), not by a walk over all of them per shard.
    std::unordered_map<uint64_t, std::pair<PvXEvent, uint64_t>> M; // key -> (query, sequence)
    using HE = std::tuple<int64_t, uint64_t, uint64_t>;              // second, sequence, key
    std::priority_queue<HE, std::vector<HE>, std::greater<HE>> H;
    uint64_t seqn = 0;
    for (uint32_t j = 0; j < me; j++) {
        for (auto &o : v[j].orph) M.erase(o.key); // answered (or found purged) in shard j
        if (!v[j].shifts.empty()) {
            int64_t last = v[j].shifts[0].first;
            for (auto &sh : v[j].shifts) last = std::max(last, sh.first);
            const int64_t lim = last - (int64_t)c->ttl_s;
            while (!H.empty() && std::get<0>(H.top()) <= lim) {
                const HE t = H.top();
                H.pop();
                auto it = M.find(std::get<2>(t));
                if (it != M.end() && it->second.second == std::get<1>(t)) M.erase(it);
            }
        }
        for (auto &q : v[j].open) {
            M[q.key] = {q, ++seqn};
            H.push(HE{(int64_t)q.sec, seqn, q.key});
        }
    }
    if (M.empty()) return 0;
    // the earliest orphan of each key (stubs are appended in stream order, one per key and batch)
    std::unordered_map<uint64_t, const PvXEvent *> orph;
    for (auto &o : v[me].orph) orph.emplace(o.key, &o);
    std::map<uint32_t, std::array<uint64_t, 4>> add; // slot -> total, out, in, timeout
    const bool quant = c->dns_groups & PV_DNS_QUANTILES;
    for (auto &kv : M) {
        const PvXEvent &qe = kv.second.first;
        const int ps = purge_shift(c->dns_shifts, c->ttl_s, qe.sec);
        auto it = orph.find(kv.first);
        if (it != orph.end() && (ps < 0 || it->second->sec < c->dns_shifts[ps].first)) {
            const PvXEvent &r = *it->second;
            const uint32_t slot = r.pad & 0x3f;
            const bool rdeep = !(r.pad & 0x40); // a response that is not deep: counts only
            const bool kept = (r.pad & 0x80) && in_dns_window(c, slot);
            // pv_xact_resolve's pairing arithmetic (timespec_diff, TransactionManager.h:24-37)
            int64_t dsec = r.sec > qe.sec ? r.sec - qe.sec : qe.sec - r.sec;
            int64_t dnsec = (int64_t)r.nsec - (int64_t)qe.nsec;
            if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
            const bool timed_out = dsec > (int64_t)c->ttl_s ||
                                   (dsec == (int64_t)c->ttl_s && ((double)dnsec / 1.0e6) >= (double)c->ttl_ms);
            auto &a = add[slot];
            if (timed_out) {
                if (kept) a[3]++;
                continue;
            }
            const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
            if (kept) {
                a[0]++;
                if (r.dir == 0) a[1]++;
                else if (r.dir == 1) a[2]++;
            }
            // sharded top_slow: the edge pair is a candidate like any valid transaction (its
            // response record was kept with the stub)
            const size_t oi = (size_t)(it->second - v[me].orph.data());
            if (c->slow_defer && oi < c->sorph.size()) {
                pv_ctx::SlowCand sc = c->sorph[oi];
                if (quant && rdeep && r.dir < 2)
                    c->slow_xv.push_back({sc.ord, PvXValue{us, 0, r.dir == 0 ? (uint32_t)XV_FROM_US : (uint32_t)XV_TO_US}});
                if (kept && rdeep && r.dir < 2) {
                    sc.us = us;
                    sc.dir = r.dir;
                    c->scands.push_back(sc);
                }
            }
            if (quant && rdeep && in_dns_window(c, slot)) {
                const uint32_t sg = slot | (c->gen[slot] << 8);
                if (r.dir == 0) c->xvals_host.push_back(PvXValue{us, sg, XV_FROM_US});
                else if (r.dir == 1) c->xvals_host.push_back(PvXValue{us, sg, XV_TO_US});
                if (qe.len && kept) {
                    const double ratio = (double)r.len / (double)qe.len;
                    uint64_t bits;
                    memcpy(&bits, &ratio, 8);
                    c->xvals_host.push_back(PvXValue{bits, sg, XV_RATIO});
                }
            }
        } else if (ps >= 0) {
            const uint32_t slot = c->dns_shifts[ps].second;
            if (in_dns_window(c, slot)) add[slot][3]++;
        }
    }
    for (auto &kv : add) {
        const uint64_t a4[4] = {kv.second[0], kv.second[1], kv.second[2], kv.second[3]};
        if (int rc = add_dns_words(c, kv.first, a4)) return rc;
    }
    return 0;
}

// Sharded runs, in rank order (pv_set_slow_defer): `in` holds the DNS queries the earlier shards
// leave open at this shard's start (the previous rank's *out); each meets the first event of its
// key in this shard as TransactionManager would (libs/visor_transaction/TransactionManager.h:51-106):
// a response pairs with it (valid or timed out), a query overwrites it, a DNS shift of this shard
// at or after ttl + its start purges it first (a time-out there, DnsStreamHandler.h:252-267);
// the rest stay open. *out: those, and this shard's own queries open at its end (pv_free).
int pv_edge_carry(pv_ctx *c, const uint8_t *in, size_t in_bytes, uint8_t **out, size_t *out_bytes)
{
    mark_merged(c, "pv_edge_carry");
    *out = nullptr;
    *out_bytes = 0;
    if (!c->slow_defer) return c->fail(PV_EINVAL, "pv_edge_carry needs pv_set_slow_defer");
    if (!c->dns2_groups && in_bytes % sizeof(PvXEvent)) return c->fail(PV_EINVAL, "malformed open-query buffer");
    if (int rc = sync_xvals(c)) return rc;
    if (c->xv_local_end == SIZE_MAX) c->xv_local_end = c->xvals_host.size();
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    if (c->dns2_groups) return edge_carry2(c, in, in_bytes, out, out_bytes);
    std::unordered_map<uint64_t, size_t> first;
    edge_first_stubs(c, in, in_bytes / sizeof(PvXEvent), sizeof(PvXEvent), first);
    const uint64_t live = c->dns.ordinal;
    auto in_win = [&](uint64_t ord) { return ord <= live && ord + c->dns.slots.size() > live; };
    const bool quant = c->dns_groups & PV_DNS_QUANTILES;
    std::map<uint32_t, std::array<uint64_t, 4>> add; // slot -> total, out, in, timeout
    std::vector<PvXEvent> keep;
    const size_t nin = in_bytes / sizeof(PvXEvent);
    for (size_t k = 0; k < nin; k++) {
        PvXEvent qe;
        memcpy(&qe, in + k * sizeof(PvXEvent), sizeof qe);
        int ps = -1;
        for (size_t i = 0; i < c->dns_shift_ord.size(); i++)
            if (c->dns_shift_ord[i].first >= (int64_t)c->ttl_s + qe.sec) { ps = (int)i; break; }
        auto purged = [&]() {
            const uint64_t o = c->dns_shift_ord[ps].second;
            if (in_win(o)) add[c->dns.slots[live - o]][3]++;
        };
        auto it = first.find(qe.key);
        if (it == first.end()) {
            if (ps >= 0) purged();
            else keep.push_back(qe);
            continue;
        }
        const pv_ctx::EdgeStub &st = c->stubs[it->second];
        if (ps >= 0 && st.ord >= c->dns_shift_ord[ps].second) { purged(); continue; } // purged before its key's next event
        if (!st.e.qr) continue;                                                          // overwritten by a new query
        const PvXEvent &r = st.e;
        const bool kept = (r.pad & 0x80) && in_win(st.ord);
        const uint32_t slot = r.pad & 0x3f;
        const bool rdeep = !(r.pad & 0x40); // a response that is not deep: counts only
        int64_t dsec = r.sec > qe.sec ? r.sec - qe.sec : qe.sec - r.sec;
        int64_t dnsec = (int64_t)r.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        const bool timed_out = dsec > (int64_t)c->ttl_s || (dsec == (int64_t)c->ttl_s && ((double)dnsec / 1.0e6) >= (double)c->ttl_ms);
        if (timed_out) { if (kept) add[slot][3]++; continue; }
        const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        if (kept) {
            auto &a = add[slot];
            a[0]++;
            if (r.dir == 0) a[1]++;
            else if (r.dir == 1) a[2]++;
        }
        if (quant && rdeep && r.dir < 2) c->slow_xv.push_back({st.ord, PvXValue{us, 0, r.dir == 0 ? (uint32_t)XV_FROM_US : (uint32_t)XV_TO_US}});
        if (quant && rdeep && in_win(st.ord)) {
            const uint32_t sg = slot | (c->gen[slot] << 8);
            if (r.dir < 2) c->xvals_host.push_back(PvXValue{us, sg, r.dir == 0 ? (uint32_t)XV_FROM_US : (uint32_t)XV_TO_US});
            if (qe.len && kept) {
                const double ratio = (double)r.len / (double)qe.len;
                uint64_t bits;
                memcpy(&bits, &ratio, 8);
                c->xvals_host.push_back(PvXValue{bits, sg, XV_RATIO});
            }
        }
        if (kept && rdeep && r.dir < 2 && st.cand >= 0) {
            pv_ctx::SlowCand sc = c->sorph[(size_t)st.cand];
            sc.us = us;
            sc.dir = r.dir;
            c->scands.push_back(sc);
        }
    }
    for (auto &kv : add) {
        const uint64_t a4[4] = {kv.second[0], kv.second[1], kv.second[2], kv.second[3]};
        if (int rc = add_dns_words(c, kv.first, a4)) return rc;
    }
    // this shard's own open queries (the carried list, latest event per key)
    if (c->n_pend) {
        std::vector<PvXEvent> pend;
        std::vector<uint64_t> pk;
        if (int rc = read_carried(c, pend, pk)) return rc;
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(pend.size() * 2);
        for (size_t i = 0; i < pend.size(); i++) {
            auto it = last.find(pend[i].key);
            if (it == last.end() || (uint32_t)pk[i] >= (uint32_t)pk[it->second]) last[pend[i].key] = i;
        }
        for (auto &kv : last) keep.push_back(pend[kv.second]);
    }
    *out_bytes = keep.size() * sizeof(PvXEvent);
    *out = (uint8_t *)malloc(*out_bytes ? *out_bytes : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "out of host memory");
    if (!keep.empty()) memcpy(*out, keep.data(), *out_bytes);
    return 0;
}

int pv_set_end_of_capture(pv_ctx *c, int on)
{
    std::lock_guard<std::mutex> g(c->mu);
    c->eoc_armed = on != 0;
    return 0;
}

int pv_merge_hints(pv_ctx *c, uint64_t *open_queries, uint64_t *xact_values)
{
    if (int rc = sync_xvals(c)) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    *open_queries = c->n_pend;
    *xact_values = c->xvals_host.size() + c->slow_xv.size() + c->scands.size();
    return 0;
}

int pv_set_slow_defer(pv_ctx *c, int defer)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (c->records_seen) return c->fail(PV_EINVAL, "set the slow-transaction mode before the first batch");
    if (defer && c->dns2_groups && !c->d_orph_ord) {
        // DNS v2 stubs carry their first-occurrence order (an edge pair's qname CPC order)
        hipSetDevice(c->device);
        hipError_t e;
        if (!hip_ok(e = hipMalloc(&c->d_orph_ord, (size_t)c->orph_cap * 8))) return c->hipfail(e, "stub orders");
    }
    c->slow_defer = defer != 0;
    return 0;
}

// This rank's own transaction times per DNS period ordinal: (ordinal u32, kind u32, value u64)
// records of kinds XV_FROM_US / XV_TO_US (DNS v2: XV2_TIME + transaction direction). Call before
// pv_values_merge (which appends the other ranks' values).
int pv_slow_values_export(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = sync_xvals(c)) return rc;
    std::vector<uint8_t> o;
    auto put = [&](uint32_t ord, const PvXValue &v) {
        const size_t p = o.size();
        o.resize(p + 16);
        memcpy(&o[p], &ord, 4);
        memcpy(&o[p + 4], &v.kind, 4);
        memcpy(&o[p + 8], &v.bits, 8);
    };
    const size_t nloc = std::min(c->xv_local_end, c->xvals_host.size());
    for (size_t i = 0; i < nloc; i++) {
        const PvXValue &v = c->xvals_host[i];
        if (v.kind != XV_FROM_US && v.kind != XV_TO_US && (v.kind < XV2_TIME || v.kind >= XV2_TIME + 3)) continue;
        auto it = c->sg_ord.find(v.slot);
        if (it != c->sg_ord.end()) put((uint32_t)it->second, v);
    }
    for (auto &ev : c->slow_xv) put((uint32_t)ev.first, ev.second);
    *bytes = o.size();
    *buf = (uint8_t *)malloc(o.size() ? o.size() : 1);
    if (!o.empty()) memcpy(*buf, o.data(), o.size());
    return 0;
}

// Every rank's pv_slow_values_export (bufs[0..nranks)): the slow thresholds of each period of
// the live DNS window over the whole stream (DnsMetricsManager::on_period_shift: at each shift
// the p90 of the bucket that closed, kept when it had no value; 0 before the first), then this
// rank's deferred candidates of those periods checked against them and counted into the
// periods' top_slow tables (DnsMetricsBucket::new_dns_transaction, dns/v1/DnsStreamHandler.cpp:
// 1121-1136). Call before the top-N exchange.
int slow_apply(pv_ctx *c, const std::vector<float> thr[5]);
int pv_slow_finish(pv_ctx *c, const uint8_t *const *bufs, const size_t *sizes, uint32_t nranks)
{
    mark_merged(c, "pv_slow_finish");
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (!c->slow_defer) return c->fail(PV_EINVAL, "pv_slow_finish without pv_set_slow_defer");
    // thresholds come from the quantile sketches: none without the quantiles group (v1) or the
    // transaction-times group (DNS v2, per transaction direction)
    const bool v2 = c->dns2_groups != 0;
    if (!c->started) return 0;
    if (v2 ? !(c->dns2_groups & PV_DNS2_XACT_TIMES)
           : (!(c->dns_groups & PV_DNS_QUANTILES) || !(c->dns_groups & PV_DNS_TRANSACTIONS)))
        return 0;
    // merged values per ordinal: [0] from, [1] to (v1); [2 + d] DNS v2 direction d
    constexpr int NK = 5;
    std::map<uint64_t, std::vector<uint64_t>> vals[NK];
    for (uint32_t r = 0; r < nranks; r++) {
        if (sizes[r] % 16) return c->fail(PV_EINVAL, "malformed slow-value buffer of rank %u", r);
        for (size_t p = 0; p < sizes[r]; p += 16) {
            uint32_t ord, kind;
            uint64_t bits;
            memcpy(&ord, bufs[r] + p, 4);
            memcpy(&kind, bufs[r] + p + 4, 4);
            memcpy(&bits, bufs[r] + p + 8, 8);
            if (kind == XV_FROM_US || kind == XV_TO_US) vals[kind == XV_TO_US][ord].push_back(bits);
            else if (kind >= XV2_TIME && kind < XV2_TIME + 3) vals[2 + kind - XV2_TIME][ord].push_back(bits);
        }
    }
    // thresholds of every ordinal up to the live one
    const uint64_t live = c->dns.ordinal;
    std::vector<float> thr[NK];
    for (int k = 0; k < NK; k++) {
        thr[k].assign(live + 1, 0.0f);
        float t = 0.0f;
        for (uint64_t o = 1; o <= live; o++) {
            auto it = vals[k].find(o - 1);
            if (it != vals[k].end() && !it->second.empty()) t = (float)quantile_at(it->second, 0.90);
            thr[k][o] = t;
        }
    }
    return slow_apply(c, thr);
}

// pv_slow_finish without shipping the values: each ordinal's p90 by the distributed selection
int slow_select(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (!c->slow_defer) return c->fail(PV_EINVAL, "pv_slow_finish without pv_set_slow_defer");
    const bool v2 = c->dns2_groups != 0;
    // (a collective: every rank takes part, even one with nothing to judge)
    const bool want = c->started && (v2 ? (c->dns2_groups & PV_DNS2_XACT_TIMES) != 0
                                        : ((c->dns_groups & PV_DNS_QUANTILES) && (c->dns_groups & PV_DNS_TRANSACTIONS)));
    if (int rc = sync_xvals(c)) return rc;
    constexpr int NK = 5;
    // the ordinals: every rank's windows hold the same (global period plan)
    const uint64_t live = c->dns.ordinal;
    std::vector<std::vector<uint64_t>> groups((size_t)NK * (live + 1));
    auto kind_of = [](uint32_t kind) {
        return kind == XV_FROM_US ? 0 : kind == XV_TO_US ? 1 : (kind >= XV2_TIME && kind < XV2_TIME + 3) ? 2 + (int)(kind - XV2_TIME) : -1;
    };
    auto put = [&](uint64_t ord, const PvXValue &v) {
        const int k = kind_of(v.kind);
        if (k >= 0 && ord <= live) groups[(size_t)k * (live + 1) + ord].push_back(v.bits);
    };
    const size_t nloc = std::min(c->xv_local_end, c->xvals_host.size());
    for (size_t i = 0; i < nloc; i++) {
        auto it = c->sg_ord.find(c->xvals_host[i].slot);
        if (it != c->sg_ord.end()) put(it->second, c->xvals_host[i]);
    }
    for (auto &ev : c->slow_xv) put(ev.first, ev.second);
    std::vector<std::vector<double>> fr(groups.size(), std::vector<double>{0.90});
    std::vector<XParts> gparts(groups.size());
    for (size_t i = 0; i < groups.size(); i++) {
        std::sort(groups[i].begin(), groups[i].end());
        gparts[i].push_back(&groups[i]);
    }
    std::vector<uint64_t> n;
    std::vector<std::vector<uint64_t>> q;
    if (int rc = x_select(c, ar, user, gparts, fr, n, q)) return rc;
    if (!want) return 0;
    std::vector<float> thr[NK];
    for (int k = 0; k < NK; k++) {
        thr[k].assign(live + 1, 0.0f);
        float t = 0.0f;
        for (uint64_t o = 1; o <= live; o++) {
            const size_t gi = (size_t)k * (live + 1) + (o - 1);
            if (n[gi]) t = (float)q[gi][0];
            thr[k][o] = t;
        }
    }
    return slow_apply(c, thr);
}

int pv_slow_x_finish(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    mark_merged(c, "pv_slow_x_finish");
    if (!ar) return c->fail(PV_EINVAL, "no all-reduce callback");
    return slow_select(c, ar, user);
}

int pv_comm_slow_finish(pv_ctx *c)
{
    mark_merged(c, "pv_comm_slow_finish");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    return slow_select(c, nullptr, nullptr);
}

// this rank's deferred slow candidates against the thresholds of every ordinal (thr[k][ord]:
// [0] from, [1] to (v1), [2 + d] DNS v2 direction d), counted into the periods' top_slow tables
// (the caller holds c->mu)
int slow_apply(pv_ctx *c, const std::vector<float> thr[5])
{
    const uint64_t live = c->dns.ordinal;
    // the window's periods: ordinal -> slot
    std::map<uint64_t, uint32_t> win;
    for (size_t i = 0; i < c->dns.slots.size(); i++) win[live - i] = c->dns.slots[i];
    std::vector<pv_ctx::SlowCand> sel;
    for (auto &sc : c->scands) {
        if (!win.count(sc.ord) || sc.ord > live) continue;
        // v1 dir 0 (toHost): from, 1 (fromHost): to; DNS v2 4 + transaction direction
        const float t = sc.dir >= 4 ? thr[2 + sc.dir - 4][sc.ord] : thr[sc.dir == 1][sc.ord];
        if (t > 0.0f && (float)sc.us >= t) sel.push_back(sc);
    }
    if (sel.empty()) return 0;
    // mini blobs (Ethernet records, TCP message records) and the valid list, by groups of at
    // most PV_MAX_SHIFTS + 1 periods (the resolve parameters' period arrays)
    std::vector<uint64_t> ords;
    for (auto &kv : win) ords.push_back(kv.first);
    for (size_t g0 = 0; g0 < ords.size(); g0 += PV_MAX_SHIFTS + 1) {
        const size_t g1 = std::min(ords.size(), g0 + PV_MAX_SHIFTS + 1);
        std::vector<uint8_t> blob[2];
        std::vector<uint32_t> offs[2];
        std::vector<PvXValid> valid;
        for (auto &sc : sel) {
            auto it = std::find(ords.begin() + g0, ords.begin() + g1, sc.ord);
            if (it == ords.begin() + g1) continue;
            const uint8_t *rec = c->sstore.data() + sc.off;
            uint32_t cap;
            memcpy(&cap, rec + 8, 4);
            const uint32_t sz = (16 + cap + 3) & ~3u;
            offs[sc.tcp].push_back((uint32_t)blob[sc.tcp].size());
            blob[sc.tcp].insert(blob[sc.tcp].end(), rec, rec + sz);
            PvXValid v{};
            v.idx = (uint32_t)(offs[sc.tcp].size() - 1) | (sc.tcp ? PV_TCP_IDX : 0u);
            v.period = (uint8_t)(it - (ords.begin() + g0));
            v.dir = sc.dir;
            v.us = sc.us;
            valid.push_back(v);
        }
        if (valid.empty()) continue;
        for (int k = 0; k < 2; k++) blob[k].resize(blob[k].size() + PV_RECS_PAD, 0);
        hipError_t e;
        uint8_t *d_blob[2] = {nullptr, nullptr};
        uint32_t *d_offs[2] = {nullptr, nullptr};
        PvXValid *d_valid = nullptr;
        struct Free { void *p[5]; ~Free() { for (void *q : p) if (q) hipFree(q); } } fr{{nullptr, nullptr, nullptr, nullptr, nullptr}};
        for (int k = 0; k < 2; k++) {
            if (!hip_ok(e = hipMalloc(&d_blob[k], blob[k].size())) || !hip_ok(e = hipMalloc(&d_offs[k], (offs[k].size() + 1) * 4)))
                return c->hipfail(e, "slow finish");
            fr.p[2 * k] = d_blob[k];
            fr.p[2 * k + 1] = d_offs[k];
            if (!hip_ok(e = hipMemcpy(d_blob[k], blob[k].data(), blob[k].size(), hipMemcpyHostToDevice)) ||
                (!offs[k].empty() && !hip_ok(e = hipMemcpy(d_offs[k], offs[k].data(), offs[k].size() * 4, hipMemcpyHostToDevice))))
                return c->hipfail(e, "slow finish");
        }
        if (!hip_ok(e = hipMalloc(&d_valid, valid.size() * sizeof(PvXValid))) ||
            !hip_ok(e = hipMemcpy(d_valid, valid.data(), valid.size() * sizeof(PvXValid), hipMemcpyHostToDevice)))
            return c->hipfail(e, "slow finish");
        fr.p[4] = d_valid;
        PvParams P;
        params_common(c, P, d_blob[0], d_offs[0], offs[0].size());
        P.sum = c->d_sum;
        P.cpc = c->d_cpc;
        P.tkeys = c->d_tkeys;
        P.tcnt = c->d_tcnt;
        P.taux = c->d_taux;
        P.tcap_log2 = c->tcap_log2;
        P.reg_log2 = c->reg_log2;
        P.arena = c->d_arena;
        P.arena_top = c->d_arena_top;
        P.arena_cap = c->arena_cap;
        P.tab_live = c->d_tab_live; // global_add counts the entries it creates
        P.flags = c->d_status + ST_FLAGS;
        PvXactParams X;
        memset(&X, 0, sizeof X);
        for (size_t j = g0; j < g1; j++) {
            const uint32_t k = (uint32_t)(j - g0);
            P.dslot_of[k] = win[ords[j]];
            X.thr_from[k] = thr[0][ords[j]];
            X.thr_to[k] = thr[1][ords[j]];
            for (int d = 0; d < 3; d++) X.thr2[k][d] = thr[2 + d][ords[j]];
            c->dns.clean[P.dslot_of[k]] = false;
        }
        X.P = P;
        X.valid = d_valid;
        X.trecs = d_blob[1];
        X.toffs = d_offs[1];
        flush_fills(c);
        *c->h_xparams = X;
        if (!hip_ok(e = hipMemcpyAsync(c->d_xparams, c->h_xparams, sizeof X, hipMemcpyHostToDevice, c->stream)))
            return c->hipfail(e, "slow finish");
        hipLaunchKernelGGL(pv_xact_slow, dim3((uint32_t)((valid.size() + 255) / 256)), dim3(256), 0, c->stream,
                           (const PvXactParams *)c->d_xparams, (uint32_t)valid.size());
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "pv_xact_slow");
    }
    uint32_t flags = 0;
    hipError_t e;
    if (!hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
    return 0;
}

// Quantile inputs (transaction values) of the live window, exchanged so every rank's
// quantiles cover the whole stream: (slot, kind, bits) records.
int pv_values_export(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = sync_xvals(c)) return rc;
    std::vector<uint8_t> o;
    for (auto &v : c->xvals_host) {
        const uint32_t slot = v.slot & 0xff;
        if (slot >= PV_SLOTS || (v.slot >> 8) != c->gen[slot] || !in_dns_window(c, slot)) continue;
        const size_t p = o.size();
        o.resize(p + 16);
        memcpy(&o[p], &v.bits, 8);
        memcpy(&o[p + 8], &slot, 4);
        memcpy(&o[p + 12], &v.kind, 4);
    }
    *bytes = o.size();
    *buf = (uint8_t *)malloc(o.size() ? o.size() : 1);
    if (!o.empty()) memcpy(*buf, o.data(), o.size());
    return 0;
}

int pv_values_merge(pv_ctx *c, const uint8_t *buf, size_t bytes)
{
    mark_merged(c, "pv_values_merge");
    std::lock_guard<std::mutex> g(c->mu);
    if (bytes % 16) return c->fail(PV_EINVAL, "malformed value buffer");
    if (int rc = sync_xvals(c)) return rc;
    for (size_t p = 0; p < bytes; p += 16) {
        PvXValue v;
        uint32_t slot;
        memcpy(&v.bits, buf + p, 8);
        memcpy(&slot, buf + p + 8, 4);
        memcpy(&v.kind, buf + p + 12, 4);
        if (slot >= PV_SLOTS) return c->fail(PV_EINVAL, "malformed value buffer");
        v.slot = slot | (c->gen[slot] << 8);
        c->xvals_host.push_back(v);
    }
    return 0;
}

// Window identity for the merge: (slot, start second) of every live bucket of one manager
// (part 0 = Net, 1 = DNS), newest first.
int pv_window_periods(pv_ctx *c, int part, uint32_t *slots, int64_t *start_sec, uint32_t max_n, uint32_t *n)
{
    std::lock_guard<std::mutex> g(c->mu);
    const Window &w = part == PART_NET ? c->net : c->dns;
    *n = (uint32_t)w.slots.size();
    for (uint32_t i = 0; i < w.slots.size() && i < max_n; i++) {
        slots[i] = w.slots[i];
        start_sec[i] = w.meta[w.slots[i]].start_sec;
    }
    return 0;
}

// Shifts of one manager that happen outside this context's stream (a sharded run: those
// whose shifting event lies in another rank's shard), applied in order as window operations
// only: a bucket opens at each threshold second (empty here), the oldest drops out, and
// next_shift moves on. No transaction purge is counted for them here (the shard that holds
// the shifting event counts its purges through pv_edge_merge).
int pv_advance_windows(pv_ctx *c, int part, const int64_t *thresh, uint32_t n)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (part != PART_NET && part != PART_DNS) return c->fail(PV_EINVAL, "part %d", part);
    if (!c->started) return c->fail(PV_EINVAL, "pv_advance_windows before the start timestamp");
    if (c->cfg.num_periods <= 1) return 0;
    Window &w = part == PART_NET ? c->net : c->dns;
    for (uint32_t k = 0; k < n; k++) {
        if (thresh[k] < w.next_shift_sec)
            return c->fail(PV_EINVAL, "shift at %lld precedes the window's next shift %lld", (long long)thresh[k],
                           (long long)w.next_shift_sec);
        clear_part(c, part, w.slot_at(1));
        win_shift(c, w, thresh[k]);
    }
    return 0;
}

// The seconds (stream order, each once) in which a batch holds a DNS event, by pv_dns_prescan.
// A sharded run's ranks exchange these to compute the DNS manager's global shifts.
// One batch of pv_dns_event_seconds: the UDP events from the prescan bits, the DNS-over-TCP
// messages from a run of the TCP stage (which advances the TCP state: the callers reset it).
static int dns_event_seconds_batch(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                                   const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n)
{
    *n = 0;
    const uint64_t nr = info->n_records;
    if (!nr) return 0;
    if (nr > c->max_records) return c->fail(PV_ECAPACITY, "batch exceeds max_records");
    uint32_t tseg[2];
    const bool filt = c->sample_rate < 100 && c->f_flags;
    if (filt && !c->d_fbits) {
        hipError_t e;
        const size_t fw = (size_t)(c->max_records / 64 + 2);
        if (!hip_ok(e = hipMalloc(&c->d_fbits, fw * 8)) || !hip_ok(e = hipHostMalloc((void **)&c->h_fbits, fw * 8, hipHostMallocDefault)))
            return c->hipfail(e, "deep sampling filter bits");
    }
    if (int rc = dns_prescan(c, d_recs, d_offs, nr, c->stream, true, tseg, filt)) return rc;
    if (int rc = tcp_stage(c, d_recs, d_offs, nr, tseg[0], tseg[1], (uint32_t)info->first_sec, true, c->stream)) return rc;
    if (c->sample_rate < 100) {
        // the DNS manager's draws in this batch: its unfiltered events (a sharded run steps
        // each rank's generator past the earlier shards' draws, pv_sample_skip)
        uint64_t d = 0;
        for (uint64_t t = 0; t < (nr + 63) / 64; t++) d += __builtin_popcountll(c->h_dbits[t] & ~(filt ? c->h_fbits[t] : 0ull));
        uint64_t dt = c->tcp_nmsg;
        if (filt && c->tcp_nmsg) {
            if (int rc = tcp_filter_bits(c, d_recs, d_offs, nr, c->stream)) return rc;
            for (uint64_t t = 0; t < ((uint64_t)c->tcp_nmsg + 63) / 64; t++) {
                uint64_t w = c->h_tfbits[t];
                if (t == (c->tcp_nmsg - 1) / 64 && (c->tcp_nmsg & 63)) w &= (1ull << (c->tcp_nmsg & 63)) - 1;
                dt -= __builtin_popcountll(w);
            }
        }
        c->plan_draws += d + dt;
    }
    // (ord, second) of every DNS event in stream order: a second's first UDP event, the messages
    std::vector<std::pair<uint64_t, int64_t>> ev;
    for (uint32_t j = 0; j < info->n_sec_changes; j++) {
        const uint64_t lo = sc_idx[j], hi = j + 1 < info->n_sec_changes ? sc_idx[j + 1] : nr;
        const uint64_t b = next_bit(c->h_dbits, lo, nr);
        if (b < hi) ev.push_back({b * 4, (int64_t)sc_sec[j]});
    }
    const size_t nu = ev.size();
    ev.insert(ev.end(), c->tcp_ords.begin(), c->tcp_ords.end());
    std::inplace_merge(ev.begin(), ev.begin() + nu, ev.end());
    c->tcp_ords.clear();
    c->tcp_nmsg = 0;
    uint32_t k = 0;
    for (auto &x : ev) {
        if (k && secs[k - 1] == x.second) continue;
        if (k >= max) return c->fail(PV_ECAPACITY, "more than %u DNS seconds", max);
        secs[k++] = x.second;
    }
    *n = k;
    return 0;
}

int pv_dns_event_seconds(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                         const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    *n = 0;
    if (c->tcp_active) return c->fail(PV_EINVAL, "pv_dns_event_seconds after DNS-over-TCP state (call it before the first batch)");
    const int rc = dns_event_seconds_batch(c, d_recs, d_offs, info, sc_idx, sc_sec, secs, max, n);
    tcp_reset(c);
    return rc;
}

} // extern "C"

// Shard cuts of a capture for a sharded run: world contiguous record ranges of about equal
// size, each cut moved to the nearest record boundary that no DNS-over-TCP flow spans (every
// flow key seen before the cut has its last packet before it), so each shard's TCP stage
// starts from the empty state a single pass holds for those flows there. A capture with a
// flow across a whole shard moves the cut past it (shards grow, some may be empty).
int pv_shard_cuts(const uint8_t *recs, size_t bytes, const uint32_t *offs, uint64_t n, uint32_t linktype, uint32_t ts_nano,
                  uint32_t world, uint64_t *cuts)
{
    if (!world) return PV_EINVAL;
    PvParams P;
    memset(&P, 0, sizeof P);
    P.linktype = linktype;
    P.ts_nano = ts_nano;
    const pvname::HostRecs R{recs, bytes};
    std::vector<uint32_t> key(n);
    std::vector<uint8_t> tcp(n, 0);
    std::unordered_map<uint32_t, uint64_t> last;
    for (uint64_t i = 0; i < n; i++) {
        if (offs[i] + 16ull > bytes) return PV_EINVAL;
        if (pvname::tcp_dns_flow(R, P, offs[i], &key[i])) {
            tcp[i] = 1;
            last[key[i]] = i;
        }
    }
    // ok[c]: no flow has packets on both sides of record boundary c
    std::vector<uint8_t> ok(n + 1, 1);
    int64_t reach = -1;
    for (uint64_t i = 0; i < n; i++) {
        if (tcp[i]) reach = std::max<int64_t>(reach, (int64_t)last[key[i]]);
        ok[i + 1] = reach <= (int64_t)i;
    }
    const uint64_t per = (n + world - 1) / world;
    cuts[0] = 0;
    for (uint32_t r = 1; r < world; r++) {
        const uint64_t lo = cuts[r - 1], ideal = std::max(lo, std::min<uint64_t>(n, (uint64_t)r * per));
        uint64_t best = n;
        for (uint64_t d = 0;; d++) {
            const bool up = ideal + d <= n, down = ideal >= lo + d;
            if (!up && !down) break;
            if (up && ok[ideal + d]) { best = ideal + d; break; }
            if (down && ok[ideal - d]) { best = ideal - d; break; }
        }
        cuts[r] = best;
    }
    cuts[world] = n;
    return 0;
}

// the Net-pass kernel the context's last span launched (the symbol rocprofv3 reports)
const char *pv_net_kernel_name(pv_ctx *c)
{
    return c ? c->net_kernel : "none";
}

// Deep sampling over a sharded stream: each manager's generator stepped past the draws the
// earlier shards make (net_draws: their records, dns_draws: their unfiltered DNS events, as
// pv_dns_event_seconds_host counts them in pv_plan_dns_draws), so every rank draws what the
// single pass draws for its events (AbstractMetricsManager::new_event, :318-323); the DNS
// manager's flag is the last of those draws (a filtered event at the shard start counts it).
// Cost: O(net_draws + dns_draws) generator steps on the calling thread (jsf32 has no jump-ahead),
// about 1 ns each; a rank calls it once, before its first batch.
int pv_sample_skip(pv_ctx *c, uint64_t net_draws, uint64_t dns_draws)
{
    if (!c) return PV_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->records_seen) return c->fail(PV_EINVAL, "pv_sample_skip after the first batch");
    if (c->sample_rate >= 100) return 0;
    Jsf32 rn, rd;
    for (uint64_t k = 0; k < net_draws; k++) rn.next();
    for (uint64_t k = 1; k < dns_draws; k++) rd.next();
    if (dns_draws) c->dns_deep_now = rd.next() % 100u < c->sample_rate; // the manager's last flag
    c->draws_net.reset(rn);
    c->draws_dns.reset(rd);
    return 0;
}

int pv_plan_dns_draws(pv_ctx *c, uint64_t *draws)
{
    *draws = c->plan_draws;
    return 0;
}
