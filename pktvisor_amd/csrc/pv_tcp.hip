// SPDX-License-Identifier: MPL-2.0
// pv_tcp.hip — DNS over TCP on the device: the TCP stage of a batch.
//
// The reference reassembles every TCP packet with PcapPlusPlus 23.09's TcpReassembly
// (third-party, not vendored; driven by PcapInputStream.cpp:75-79,254-283,429-465) and cuts
// DNS messages out of each side's byte stream with DnsTcpSessionData's 2-byte framing
// (src/handlers/dns/v1/DnsStreamHandler.cpp:337-436). Reassembly is sequential per
// connection and independent across connections, so the stage is one lane per flow:
//
//   Net pass / prescan  segments of DNS-port TCP flows (PvTcpSeg) + per-tile TCP masks
//   pv_tcp_keys + sort  (flowKey, record index) with rocPRIM: each flow's packets contiguous,
//                       in capture order
//   pv_tcp_scan         prefix maximum of TCP record seconds over the batch's tiles (the
//                       30 s connection timeout of PcapInputStream's LRU needs "a TCP packet
//                       at >= t + 30 before this one")
//   pv_tcp_lookup/insert the flow's carried entry in the device flow table
//   pv_tcp_flow         TcpReassembly::reassemblePacket, checkOutOfOrderFragments,
//                       handleFinOrRst, closeConnectionInternal and the session framing,
//                       over the flow's packets; every complete message is written as a
//                       message record (pv_layout.h) and a DnsMsg work item
//   pv_tcp_migrate      carried bytes of flows with no packet in this batch move to the
//                       new carry arena
// The messages then go through the DNS pass like UDP datagrams (pv_dns_tcp).
//
// Exact LRU mode (pv_set_tcp_exact_lru, implied by tcp_packet_reassembly_cache_limit): every TCP
// packet is a segment; a dry run of pv_tcp_flow records each segment's LRU events, the host
// replays PcapInputStream's LRU list over them in capture order (puts with ConnectionData's
// endTime, 0 until a connection's second packet; after every TCP packet at most 100 time-outs
// from the tail; evictions past the limit) and the real run closes the flows it closed, with
// close-only segments for flows that have no packet in the batch (pv_host.cpp tcp_lru_replay).
// Default mode: a connection times out lazily at its next packet, once a TCP packet 30 s after
// its last put's second came before it; the LRU holds the DNS-port connections only. The two
// differ for a connection whose last put carried the zero endTime (a first packet with data: a
// capture without the handshake), which the reference closes as soon as it reaches the LRU's
// tail, and when more than 100 connections time out at one packet. Not modelled in either: the
// closed-connection purge (wall clock in PcapPlusPlus), the puts of data that closing an evicted
// connection flushes. The flush of open connections at the end of a capture is pv_tcp_eoc's
// segments in the final batch (pv_set_end_of_capture).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include "pv_layout.h"

#define PV_C __attribute__((address_space(4)))
#define PV_CREF(T) const PV_C T &

namespace {

__device__ __forceinline__ uint32_t fmix32(uint32_t h)
{
    h ^= h >> 16; h *= 0x85ebca6bu;
    h ^= h >> 13; h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ bool seq_lt(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }
__device__ __forceinline__ bool seq_gt(uint32_t a, uint32_t b) { return (int32_t)(b - a) < 0; }
__device__ __forceinline__ bool dns_port(uint32_t p) { return p == 53 || p == 5353 || p == 5355 || p == 53000; }
__device__ __forceinline__ bool run_start(PV_CREF(PvTcpParams) T, uint32_t j)
{
    return j == 0 || (T.skey[j] >> 32) != (T.skey[j - 1] >> 32);
}
#define PV_RUN_NONE 0xffffffffu
#define PV_RUN_NEW 0xfffffffeu

// an entry whose connection closed (or timed out) PV_TCP_RECLAIM seconds ago, or one that never
// started a connection (a run of ignored packets)
__device__ __forceinline__ bool reclaimable(const PV_G PvTcpFlow &f, uint32_t now)
{
    if (!f.live) return true;
    if (f.closed) return f.close_sec + PV_TCP_RECLAIM <= now;
    return f.lru_sec + PV_TCP_TIMEOUT + PV_TCP_RECLAIM <= now;
}

// ---- per-flow working state
#define PV_NOREC 0xffffffffu
struct Flow {
    PvTcpFlow f;
    uint32_t head[2], cnt[2]; // fragment lists (node indices)
    uint32_t rec[2], res[2];  // message record being filled per side (arena offset, bytes reserved)
    uint32_t budget;          // bound on bytes this flow can deliver in this batch
    uint32_t fkey;
    uint32_t cur_idx, cur_dir, cur_sec, sub;
    uint32_t ev;      // PVT_EV_* of the packet being replayed (exact LRU mode's dry run)
    uint32_t put_sec; // LRU time of its last put
};

__device__ void emit_msg(PV_CREF(PvTcpParams) T, Flow &F, int s)
{
    const uint32_t size = F.f.size[s];
    const uint32_t off = F.rec[s];
    uint8_t *r = T.marena + off;
    // classic-pcap record: ts, incl_len, orig_len; raw IPv4 (total length 0), UDP
    const uint32_t incl = 28u + size;
    // UDP ports: the connection's metric port as the source, 53 as the destination, so the
    // record's ports give the metric port as a datagram's would (dns_port)
    const uint32_t pw = ((uint32_t)F.f.port >> 8) | (((uint32_t)F.f.port & 0xffu) << 8) | (53u << 24);
    const uint32_t hw[11] = {F.f.end_sec, F.f.end_usec, incl, incl, 0x00000045u, 0u, 0x00001140u, 0u, 0u, pw,
                             (((8u + size) >> 8) & 0xffu) | ((8u + size) & 0xffu) << 8};
    for (int k = 0; k < 11; k++)
        for (int b = 0; b < 4; b++) r[k * 4 + b] = (uint8_t)(hw[k] >> (8 * b));
    const uint32_t q = atomicAdd(&T.cnt[PVT_NMSG], 1u);
    if (q >= T.mq_cap) { atomicOr(&T.cnt[PVT_FLAGS], (uint32_t)PVT_F_MSGS); return; }
    T.moffs[q] = off;
    const uint32_t ord = F.cur_idx * 4u + min(F.sub, 3u);
    F.sub++;
    const uint32_t flags = F.cur_dir | (F.f.v6 ? 4u : 0u);
    uint4 *d = reinterpret_cast<uint4 *>(T.mq + (uint64_t)q * 4);
    d[0] = make_uint4(q, off + PV_TCP_REC_HDR, size | (size << 16), (uint32_t)F.f.port | (flags << 16));
    d[1] = make_uint4(F.fkey, F.f.end_sec, F.f.end_usec * 1000u, ord);
}

// a message record for side s once its size is known (bytes the batch can still deliver bound it)
__device__ bool start_msg(PV_CREF(PvTcpParams) T, Flow &F, int s)
{
    const uint32_t want = min((uint32_t)F.f.size[s], F.budget);
    const uint32_t bytes = (PV_TCP_REC_HDR + want + 3u) & ~3u;
    const uint32_t off = atomicAdd(&T.cnt[PVT_ARENA], bytes);
    if ((uint64_t)off + bytes > T.marena_cap) {
        atomicOr(&T.cnt[PVT_FLAGS], (uint32_t)PVT_F_ARENA);
        F.rec[s] = PV_NOREC;
        F.res[s] = 0;
        return false;
    }
    F.rec[s] = off;
    F.res[s] = want;
    return true;
}

// DnsTcpSessionData::receive_tcp_data, streaming: the 2 length bytes, then the message
// bytes straight into its record; a size below 17 makes the session invalid once 19
// bytes are buffered
__device__ void frame(PV_CREF(PvTcpParams) T, Flow &F, int s, const uint8_t *src, uint32_t n)
{
    PvTcpFlow &f = F.f;
    while (n && !f.inval[s]) {
        if (f.lenb[s] < 2) {
            const uint32_t b = *src++;
            n--;
            if (f.lenb[s] == 0) { f.size[s] = (uint16_t)(b << 8); f.lenb[s] = 1; }
            else {
                f.size[s] = (uint16_t)(f.size[s] | b);
                f.lenb[s] = 2;
                f.got[s] = 0;
                if (f.size[s] >= PV_TCP_MIN_MSG) start_msg(T, F, s);
            }
            continue;
        }
        if (f.size[s] < PV_TCP_MIN_MSG) {
            const uint32_t take = min(n, PV_TCP_MIN_MSG - f.got[s]);
            f.got[s] += take; src += take; n -= take;
            if (f.got[s] >= PV_TCP_MIN_MSG) { f.inval[s] = 1; f.lenb[s] = 0; f.got[s] = 0; }
            continue;
        }
        const uint32_t take = min(n, (uint32_t)f.size[s] - f.got[s]);
        if (F.rec[s] != PV_NOREC) {
            uint8_t *dst = T.marena + F.rec[s] + PV_TCP_REC_HDR + f.got[s];
            const uint32_t room = F.res[s] > f.got[s] ? F.res[s] - f.got[s] : 0u;
            const uint32_t cp = min(take, room);
            for (uint32_t k = 0; k < cp; k++) dst[k] = src[k];
        }
        f.got[s] += take; src += take; n -= take;
        if (f.got[s] == f.size[s]) {
            if (F.rec[s] != PV_NOREC && F.res[s] == f.size[s]) emit_msg(T, F, s);
            F.rec[s] = PV_NOREC;
            f.lenb[s] = 0;
            f.got[s] = 0;
        }
    }
}

// onMessageReady -> PcapInputStream::tcp_message_ready: the DNS handler's session (a
// tracked, i.e. DNS-port, connection), then the LRU put
__device__ void deliver(PV_CREF(PvTcpParams) T, Flow &F, int s, const uint8_t *src, uint32_t n)
{
    if (F.f.port) frame(T, F, s, src, n);
    F.f.lru_sec = F.cur_sec;
    F.put_sec = F.f.end_sec;
    F.ev |= PVT_EV_PUT;
}

__device__ uint32_t frag_new(PV_CREF(PvTcpParams) T, const uint8_t *src, uint32_t seq, uint32_t len)
{
    const uint32_t q = atomicAdd(&T.cnt[PVT_NFRAG], 1u);
    if (q >= T.frag_cap) { atomicOr(&T.cnt[PVT_FLAGS], (uint32_t)PVT_F_FRAGS); return PV_TCP_FRAG_NIL; }
    T.frags[q] = PvTcpFrag{(uint64_t)(uintptr_t)src, seq, len, PV_TCP_FRAG_NIL, 0};
    return q;
}
__device__ void frag_push(PV_CREF(PvTcpParams) T, Flow &F, int s, uint32_t q)
{
    if (q == PV_TCP_FRAG_NIL) return;
    // append at the tail (pushBack)
    if (F.head[s] == PV_TCP_FRAG_NIL) F.head[s] = q;
    else {
        uint32_t t = F.head[s];
        while (T.frags[t].next != PV_TCP_FRAG_NIL) t = T.frags[t].next;
        T.frags[t].next = q;
    }
    F.cnt[s]++;
}
__device__ void frag_unlink(PV_CREF(PvTcpParams) T, Flow &F, int s, uint32_t prev, uint32_t q)
{
    const uint32_t nx = T.frags[q].next;
    if (prev == PV_TCP_FRAG_NIL) F.head[s] = nx;
    else T.frags[prev].next = nx;
    F.cnt[s]--;
}

// TcpReassembly::checkOutOfOrderFragments
__device__ void check_ooo(PV_CREF(PvTcpParams) T, Flow &F, int s, bool clean)
{
    bool found;
    do {
        do {
            found = false;
            uint32_t prev = PV_TCP_FRAG_NIL, q = F.head[s];
            while (q != PV_TCP_FRAG_NIL) {
                const PvTcpFrag fr = T.frags[q];
                const uint32_t exp = F.f.seq[s];
                if (fr.seq == exp) {
                    F.f.seq[s] = exp + fr.len;
                    frag_unlink(T, F, s, prev, q);
                    deliver(T, F, s, (const uint8_t *)(uintptr_t)fr.src, fr.len);
                    found = true;
                    q = fr.next;
                    continue;
                }
                if (seq_lt(fr.seq, exp)) {
                    frag_unlink(T, F, s, prev, q);
                    const uint32_t nseq = fr.seq + fr.len;
                    if (seq_gt(nseq, exp)) {
                        const uint32_t nl = exp - fr.seq;
                        F.f.seq[s] += fr.len - nl;
                        deliver(T, F, s, (const uint8_t *)(uintptr_t)fr.src + nl, fr.len - nl);
                        found = true;
                    }
                    q = fr.next;
                    continue;
                }
                prev = q;
                q = fr.next;
            }
        } while (found);
        if (!clean && F.cnt[s] <= PV_TCP_MAX_OOO) return;
        // missing data: the fragment with the lowest sequence, behind "[N bytes missing]"
        uint32_t best = PV_TCP_FRAG_NIL, bprev = PV_TCP_FRAG_NIL, prev = PV_TCP_FRAG_NIL;
        uint32_t closest = 0xffffffffu;
        for (uint32_t q = F.head[s]; q != PV_TCP_FRAG_NIL; prev = q, q = T.frags[q].next)
            if (best == PV_TCP_FRAG_NIL || seq_lt(T.frags[q].seq, closest)) { closest = T.frags[q].seq; best = q; bprev = prev; }
        if (best != PV_TCP_FRAG_NIL) {
            const PvTcpFrag fr = T.frags[best];
            frag_unlink(T, F, s, bprev, best);
            const uint32_t missing = fr.seq - F.f.seq[s];
            F.f.seq[s] = fr.seq + fr.len;
            // prepareMissingDataMessage: "[" << missing << " bytes missing]", one callback with the data
            uint8_t txt[32];
            uint32_t n = 0, digits[10], nd = 0, v = missing;
            do { digits[nd++] = v % 10u; v /= 10u; } while (v);
            txt[n++] = '[';
            while (nd) txt[n++] = (uint8_t)('0' + digits[--nd]);
            const char *tail = " bytes missing]";
            for (int k = 0; tail[k]; k++) txt[n++] = (uint8_t)tail[k];
            if (F.f.port) {
                frame(T, F, s, txt, n);
                frame(T, F, s, (const uint8_t *)(uintptr_t)fr.src, fr.len);
            }
            F.f.lru_sec = F.cur_sec;
            F.put_sec = F.f.end_sec;
            F.ev |= PVT_EV_PUT;
            found = true;
        }
    } while (found);
}

// closing the connection now would deliver data (checkOutOfOrderFragments with cleanup: a held
// fragment that ends past the side's next sequence), so the close puts it into the LRU list
// once more (PcapInputStream::tcp_message_ready) before its end erases it
__device__ bool held_delivery(PV_CREF(PvTcpParams) T, const Flow &F)
{
    for (int s = 0; s < 2; s++)
        for (uint32_t q = F.head[s]; q != PV_TCP_FRAG_NIL; q = T.frags[q].next)
            if (seq_gt(T.frags[q].seq + T.frags[q].len, F.f.seq[s])) return true;
    return false;
}

// TcpReassembly::closeConnectionInternal (+ DnsStreamHandler::tcp_connection_end_cb)
__device__ void close_conn(PV_CREF(PvTcpParams) T, Flow &F, uint32_t when)
{
    check_ooo(T, F, 0, true);
    check_ooo(T, F, 1, true);
    F.f.closed = 1;
    F.f.close_sec = when;
    F.ev |= PVT_EV_CLOSE;
    F.f.port = 0; // untracked: the sessions are gone
    for (int s = 0; s < 2; s++) { F.f.inval[s] = 0; F.f.lenb[s] = 0; F.f.size[s] = 0; F.f.got[s] = 0; F.rec[s] = PV_NOREC; }
}

// TcpReassembly::handleFinOrRst
__device__ void fin_rst(PV_CREF(PvTcpParams) T, Flow &F, int s, bool rst)
{
    if (F.f.fin[s]) return;
    F.f.fin[s] = 1;
    if (F.f.fin[1 - s] || rst) close_conn(T, F, F.cur_sec);
    else check_ooo(T, F, s, true);
}

// the latest TCP record second (+1; 0: none) before record i of the batch, earlier batches included
__device__ uint32_t lt_before(PV_CREF(PvTcpParams) T, uint32_t i)
{
    const uint32_t t = i >> 6, lane = i & 63;
    uint32_t v = T.tpm[t];
    const uint64_t m = T.tmask[t] & ((1ull << lane) - 1);
    if (m) {
        const uint32_t h = 63 - __builtin_clzll(m);
        const uint32_t r = (t << 6) + h;
        const uint32_t sec = *reinterpret_cast<const uint32_t *>(T.recs + T.offs[r]);
        v = max(v, sec + 1);
    }
    return v;
}

// TcpReassembly::reassemblePacket for one packet of the flow
__device__ void packet(PV_CREF(PvTcpParams) T, Flow &F, const PvTcpSeg &g)
{
    if (g.idx != F.cur_idx) F.sub = 0;
    F.cur_idx = g.idx;
    F.cur_dir = g.dirv6 & 3;
    F.cur_sec = g.sec;
    PvTcpFlow &f = F.f;
    // Ignore_PacketWithNoData / no TCP layer, before the connection lookup; a close-only segment
    if (g.flags & (PV_TF_NODATA | PV_TF_CLOSE)) return;
    if (!T.exact && f.live && !f.closed) {
        // PcapInputStream's LRU cleanup after an earlier TCP packet at >= last put + 30 s
        const uint32_t lt = lt_before(T, g.idx);
        if (lt && lt - 1 >= f.lru_sec + PV_TCP_TIMEOUT) {
            close_conn(T, F, f.lru_sec + PV_TCP_TIMEOUT);
            F.ev = PVT_EV_TIMEOUT;
        }
    }
    if (f.closed) return; // Ignore_PacketOfClosedFlow
    const bool fin = g.flags & PV_TF_FIN, syn = g.flags & PV_TF_SYN, rst = g.flags & PV_TF_RST;
    const uint32_t plen = g.plen;
    const uint8_t *pl = T.recs + g.poff;
    if (!f.live) {
        // a new connection: onConnectionStart -> tcp_connection_start (tracking, LRU put)
        f.live = 1;
        f.sport = g.sport;
        f.dport = g.dport;
        f.v6 = (g.dirv6 >> 2) & 1;
        f.port = dns_port(g.dport) ? g.sport : (dns_port(g.sport) ? g.dport : 0);
        f.end_sec = f.end_usec = 0;
        f.prev = -1;
        f.lru_sec = g.sec;
        F.put_sec = g.sec;
        F.ev |= PVT_EV_NEW;
    } else if (g.sec > f.end_sec || (g.sec == f.end_sec && g.usec > f.end_usec)) {
        f.end_sec = g.sec;
        f.end_usec = g.usec;
    }
    int s;
    bool first = false;
    if (f.nsides < 2 && !(f.nsides == 1 && f.ep[0] == g.ep)) {
        s = f.nsides++;
        f.ep[s] = g.ep;
        first = true;
    } else if (f.ep[0] == g.ep) s = 0;
    else if (f.nsides == 2 && f.ep[1] == g.ep) s = 1;
    else return; // Error_PacketDoesNotMatchFlow
    if (f.fin[s]) return;
    if ((fin || rst) && plen == 0) { fin_rst(T, F, s, rst); return; }
    if (f.prev != -1 && f.prev != s) check_ooo(T, F, f.prev, true);
    f.prev = (int8_t)s;
    if (first) {
        f.seq[s] = g.seq + plen + (syn ? 1u : 0u);
        if (plen) deliver(T, F, s, pl, plen);
    } else if (seq_lt(g.seq, f.seq[s])) {
        const uint32_t nseq = g.seq + plen;
        if (seq_gt(nseq, f.seq[s])) {
            const uint32_t nl = f.seq[s] - g.seq;
            f.seq[s] += plen - nl;
            deliver(T, F, s, pl + nl, plen - nl);
        }
    } else if (g.seq == f.seq[s]) {
        if (plen) {
            f.seq[s] += plen + (syn ? 1u : 0u);
            deliver(T, F, s, pl, plen);
            check_ooo(T, F, s, false);
        }
    } else if (plen) {
        frag_push(T, F, s, frag_new(T, pl, g.seq, plen));
        if (F.cnt[s] > PV_TCP_MAX_OOO) check_ooo(T, F, s, true);
    }
    if (fin || rst) fin_rst(T, F, s, rst);
}

__device__ __forceinline__ uint32_t rd32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

} // namespace

// sort keys of the batch's segments: flowKey, then capture order
extern "C" __global__ void pv_tcp_keys(const PvTcpSeg *seg, uint32_t n, uint64_t *key, uint32_t *val)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const PvTcpSeg g = seg[j];
    key[j] = ((uint64_t)g.fkey << 32) | g.idx;
    val[j] = j;
}

// tpm[t] = 1 + the latest TCP record second before tile t (0: none), from the tile masks;
// lt_carry holds the value past the previous batches and is advanced to this batch's end.
// One workgroup of 1024 threads, each scanning a contiguous run of tiles.
extern "C" __global__ void __launch_bounds__(1024) pv_tcp_scan(const PvTcpParams *__restrict__ Tp)
{
    PV_CREF(PvTcpParams) T = *(const PV_C PvTcpParams *)Tp;
    __shared__ uint32_t part[1024];
    const uint32_t n = T.n_tiles, per = (n + 1023) / 1024;
    const uint32_t a = min(threadIdx.x * per, n), b = min(a + per, n);
    auto tile_max = [&](uint32_t t) -> uint32_t {
        const uint64_t m = T.tmask[t];
        if (!m) return 0u;
        const uint32_t r = (t << 6) + (63 - __builtin_clzll(m));
        return *reinterpret_cast<const uint32_t *>(T.recs + T.offs[r]) + 1u;
    };
    uint32_t mx = 0;
    for (uint32_t t = a; t < b; t++) mx = max(mx, tile_max(t));
    part[threadIdx.x] = mx;
    __syncthreads();
    // exclusive prefix maximum of the run maxima (Hillis-Steele on the inclusive form)
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
        __syncthreads();
        part[threadIdx.x] = max(part[threadIdx.x], v);
        __syncthreads();
    }
    // a dry run (cache-limit replay) leaves the carried value for the run after it
    const uint32_t carry = *T.lt_carry;
    uint32_t run = max(carry, threadIdx.x ? part[threadIdx.x - 1] : 0u);
    for (uint32_t t = a; t < b; t++) {
        T.tpm[t] = run;
        run = max(run, tile_max(t));
    }
    __syncthreads();
    if (threadIdx.x == 0 && !T.dry) *T.lt_carry = max(carry, part[1023]);
}

// the flow-table entry of every run (a flow's first sorted segment): found, or PV_RUN_NEW
extern "C" __global__ void pv_tcp_lookup(const PvTcpParams *__restrict__ Tp)
{
    PV_CREF(PvTcpParams) T = *(const PV_C PvTcpParams *)Tp;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= T.n_seg) return;
    if (!run_start(T, j)) { T.run_flow[j] = PV_RUN_NONE; return; }
    const uint32_t fkey = (uint32_t)(T.skey[j] >> 32);
    const uint64_t tag = (1ull << 32) | fkey;
    const uint32_t mask = (1u << T.flow_cap_log2) - 1;
    uint32_t h = fmix32(fkey) & mask;
    for (uint32_t p = 0; p <= mask; p++, h = (h + 1) & mask) {
        const uint64_t t = T.flows[h].tag;
        if (t == tag) { T.run_flow[j] = h; T.flows[h].stage = T.stage; return; }
        if (t == 0) break;
    }
    T.run_flow[j] = PV_RUN_NEW;
}

// new entries: the first empty slot of the probe sequence, or an entry no run of this
// batch holds whose connection ended PV_TCP_RECLAIM seconds ago
extern "C" __global__ void pv_tcp_insert(const PvTcpParams *__restrict__ Tp)
{
    PV_CREF(PvTcpParams) T = *(const PV_C PvTcpParams *)Tp;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= T.n_seg || T.run_flow[j] != PV_RUN_NEW) return;
    if (T.seg[T.sval[j]].flags & PV_TF_CLOSE) { T.run_flow[j] = PV_RUN_NONE; return; } // its flow is gone
    const uint32_t fkey = (uint32_t)(T.skey[j] >> 32);
    const uint64_t tag = (1ull << 32) | fkey;
    const uint32_t mask = (1u << T.flow_cap_log2) - 1;
    uint32_t h = fmix32(fkey) & mask;
    for (uint32_t p = 0; p <= mask; p++, h = (h + 1) & mask) {
        PV_G PvTcpFlow &e = T.flows[h];
        const uint64_t t = __atomic_load_n(&e.tag, __ATOMIC_RELAXED);
        const bool take = t == 0 || (e.stage != T.stage && reclaimable(e, T.now_sec));
        if (!take) continue;
        if (atomicCAS((unsigned long long *)&e.tag, (unsigned long long)t, (unsigned long long)tag) != t) continue;
        PvTcpFlow z;
        memset(&z, 0, sizeof z);
        z.tag = tag;
        z.stage = T.stage;
        z.prev = -1;
        e = z;
        T.run_flow[j] = h;
        return;
    }
    atomicOr(&T.cnt[PVT_FLAGS], (uint32_t)PVT_F_TABLE);
    T.run_flow[j] = PV_RUN_NONE;
}

// one lane per flow of the batch: its carried state, its packets in capture order, the
// bytes it carries into the next batch
extern "C" __global__ void __launch_bounds__(256) pv_tcp_flow(const PvTcpParams *__restrict__ Tp)
{
    PV_CREF(PvTcpParams) T = *(const PV_C PvTcpParams *)Tp;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= T.n_seg) return;
    const uint32_t fi = T.run_flow[j];
    if (fi >= PV_RUN_NEW) return;
    Flow F;
    F.f = T.flows[fi];
    F.fkey = (uint32_t)(T.skey[j] >> 32);
    uint32_t je = j + 1;
    while (je < T.n_seg && (uint32_t)(T.skey[je] >> 32) == F.fkey) je++;
    F.head[0] = F.head[1] = PV_TCP_FRAG_NIL;
    F.cnt[0] = F.cnt[1] = 0;
    F.rec[0] = F.rec[1] = PV_NOREC;
    F.res[0] = F.res[1] = 0;
    F.cur_idx = 0xffffffffu;
    F.cur_dir = 2;
    F.cur_sec = 0;
    F.sub = 0;
    F.ev = 0;
    F.put_sec = 0;
    // bytes this flow can deliver in this batch: carried bytes, payloads, missing-data texts
    uint64_t budget = F.f.blob_len + 32ull * (F.f.nfrag[0] + F.f.nfrag[1]);
    for (uint32_t k = j; k < je; k++) budget += T.seg[T.sval[k]].plen + 32u;
    F.budget = (uint32_t)min<uint64_t>(budget, 0xffffffffull);
    // carried state: held message bytes, then the fragment lists
    if (F.f.blob_len) {
        const uint8_t *b = T.carry_in + F.f.blob;
        for (int s = 0; s < 2; s++) {
            if (F.f.lenb[s] == 2 && F.f.size[s] >= PV_TCP_MIN_MSG && F.f.got[s] && !F.f.inval[s]) {
                const uint32_t got = F.f.got[s];
                if (start_msg(T, F, s)) {
                    uint8_t *dst = T.marena + F.rec[s] + PV_TCP_REC_HDR;
                    for (uint32_t k = 0; k < min(got, F.res[s]); k++) dst[k] = b[k];
                }
                b += (got + 3u) & ~3u;
            }
        }
        for (int s = 0; s < 2; s++)
            for (uint32_t k = 0; k < F.f.nfrag[s]; k++) {
                const uint32_t seq = rd32(b), len = rd32(b + 4);
                frag_push(T, F, s, frag_new(T, b + 8, seq, len));
                b += 8 + ((len + 3u) & ~3u);
            }
    }
    F.f.blob_len = 0;
    F.f.nfrag[0] = F.f.nfrag[1] = 0;
    // the close the host's LRU replay decided (a time-out or an eviction after record fc_idx,
    // usually another flow's packet): closeConnection with that record's second and direction;
    // its flushed messages rank behind the record's own (sub 3)
    uint32_t fc_idx = PVT_FCLOSE_NONE, fc_sec = 0, fc_dir = 2;
    if (T.fclose) {
        const uint32_t s0 = T.sval[j];
        fc_idx = T.fclose[3 * s0]; fc_sec = T.fclose[3 * s0 + 1]; fc_dir = T.fclose[3 * s0 + 2];
    }
    auto force_close = [&]() {
        F.cur_idx = fc_idx;
        F.sub = 3;
        F.cur_sec = fc_sec;
        F.cur_dir = fc_dir;
        close_conn(T, F, fc_sec);
    };
    for (uint32_t k = j; k < je; k++) {
        const PvTcpSeg g = T.seg[T.sval[k]];
        if (fc_idx != PVT_FCLOSE_NONE && g.idx > fc_idx && F.f.live && !F.f.closed)
            force_close();
        if (g.flags & PV_TF_EOC) {
            // closeAllConnections after the capture's last record: the connection's held fragments
            // go out behind their missing-data markers, its messages at its endTime, with the
            // direction of the capture's last packet (_packet_dir_cache). A connection the default
            // mode would have timed out at a later TCP packet of another flow closes at its
            // time-out second, as it would have there.
            if (F.f.live && !F.f.closed) {
                F.cur_idx = g.idx;
                F.sub = 3;
                F.cur_sec = g.sec;
                F.cur_dir = g.dirv6 & 3;
                uint32_t when = g.sec;
                if (!T.exact) {
                    const uint32_t lt = *T.lt_carry;
                    if (lt && lt - 1 >= F.f.lru_sec + PV_TCP_TIMEOUT) when = F.f.lru_sec + PV_TCP_TIMEOUT;
                }
                close_conn(T, F, when);
            }
            continue;
        }
        F.ev = 0;
        F.put_sec = 0;
        packet(T, F, g);
        if (T.lru_ev) {
            if (!F.f.closed && held_delivery(T, F)) F.ev |= PVT_EV_HOLD;
            T.lru_ev[3 * k] = F.ev | (g.dirv6 & 3) << 8;
            T.lru_ev[3 * k + 1] = g.sec;
            T.lru_ev[3 * k + 2] = F.put_sec;
        }
    }
    if (fc_idx != PVT_FCLOSE_NONE && F.f.live && !F.f.closed) force_close();
    if (T.dry) return; // the LRU replay's dry run: flow state and carried bytes as they were
    // carry out: held message bytes (from their records) and the fragments left
    if (!F.f.closed) {
        uint32_t bytes = 0;
        for (int s = 0; s < 2; s++) {
            if (F.f.lenb[s] == 2 && F.f.size[s] >= PV_TCP_MIN_MSG && F.f.got[s] && !F.f.inval[s]) bytes += (F.f.got[s] + 3u) & ~3u;
            for (uint32_t q = F.head[s]; q != PV_TCP_FRAG_NIL; q = T.frags[q].next) bytes += 8 + ((T.frags[q].len + 3u) & ~3u);
        }
        if (bytes) {
            const uint32_t off = atomicAdd(&T.cnt[PVT_CARRY], bytes);
            if ((uint64_t)off + bytes > T.carry_cap) {
                atomicOr(&T.cnt[PVT_FLAGS], (uint32_t)PVT_F_CARRY);
            } else {
                uint8_t *o = T.carry_out + off;
                for (int s = 0; s < 2; s++) {
                    if (F.f.lenb[s] == 2 && F.f.size[s] >= PV_TCP_MIN_MSG && F.f.got[s] && !F.f.inval[s]) {
                        const uint32_t got = F.f.got[s];
                        const uint8_t *src = F.rec[s] != PV_NOREC ? T.marena + F.rec[s] + PV_TCP_REC_HDR : nullptr;
                        for (uint32_t k = 0; k < got; k++) o[k] = (src && k < F.res[s]) ? src[k] : 0;
                        o += (got + 3u) & ~3u;
                    }
                }
                for (int s = 0; s < 2; s++) {
                    for (uint32_t q = F.head[s]; q != PV_TCP_FRAG_NIL; q = T.frags[q].next) {
                        const PvTcpFrag fr = T.frags[q];
                        for (int b = 0; b < 4; b++) { o[b] = (uint8_t)(fr.seq >> (8 * b)); o[4 + b] = (uint8_t)(fr.len >> (8 * b)); }
                        const uint8_t *src = (const uint8_t *)(uintptr_t)fr.src;
                        for (uint32_t k = 0; k < fr.len; k++) o[8 + k] = src[k];
                        o += 8 + ((fr.len + 3u) & ~3u);
                    }
                    F.f.nfrag[s] = (uint16_t)min(F.cnt[s], 65535u);
                }
                F.f.blob = off;
                F.f.blob_len = bytes;
                T.clist_out[atomicAdd(&T.cnt[PVT_NCARRY], 1u)] = fi;
            }
        }
    }
    F.f.stage = T.stage;
    T.flows[fi] = F.f;
}

// TcpReassembly::closeAllConnections at the end of a capture: a close segment (PV_TF_EOC) for
// every connection that may be open after the batch, at the batch's last record (idx), the
// record's time and the direction of the capture's last packet; the TCP stage then runs them as
// its last segments. Candidates: the open entries of the flow table (threads [0, 2^flow_cap_log2))
// and the flow keys of the batch's segments (the threads after), once each (a hash set of the
// keys, at least twice the candidates in size); a close of a connection the batch closes is a
// no-op in pv_tcp_flow.
extern "C" __global__ void pv_tcp_eoc(const PvTcpParams *__restrict__ Tp, const PvTcpSeg *__restrict__ seg, uint32_t n_seg,
                                      uint64_t *__restrict__ set, uint32_t set_mask, PvTcpSeg *__restrict__ out,
                                      uint32_t *__restrict__ cnt, uint32_t idx, uint32_t sec, uint32_t usec, uint32_t dir)
{
    PV_CREF(PvTcpParams) T = *(const PV_C PvTcpParams *)Tp;
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ncap = 1u << T.flow_cap_log2;
    uint32_t fkey;
    if (h < ncap) {
        const PV_G PvTcpFlow &f = T.flows[h];
        if (!(f.tag >> 32) || !f.live || f.closed) return;
        fkey = (uint32_t)f.tag;
    } else if (h - ncap < n_seg) {
        fkey = seg[h - ncap].fkey;
    } else {
        return;
    }
    const uint64_t mine = (1ull << 32) | fkey;
    for (uint32_t slot = fmix32(fkey) & set_mask;; slot = (slot + 1) & set_mask) {
        const uint64_t prev = atomicCAS((unsigned long long *)&set[slot], 0ull, (unsigned long long)mine);
        if (prev == mine) return; // another candidate of this connection emits it
        if (prev == 0) break;
    }
    PvTcpSeg g;
    memset(&g, 0, sizeof g);
    g.idx = idx;
    g.fkey = fkey;
    g.sec = sec;
    g.usec = usec;
    g.flags = PV_TF_CLOSE | PV_TF_EOC;
    g.dirv6 = (uint8_t)dir;
    out[atomicAdd(cnt, 1u)] = g;
}

// flows that carried bytes into this batch but had no packet in it keep them: copied to
// the new carry arena
extern "C" __global__ void pv_tcp_migrate(const PvTcpParams *__restrict__ Tp)
{
    PV_CREF(PvTcpParams) T = *(const PV_C PvTcpParams *)Tp;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= T.n_clist_in) return;
    const uint32_t fi = T.clist_in[j];
    PV_G PvTcpFlow &e = T.flows[fi];
    if (e.stage == T.stage || !e.blob_len || e.closed) return;
    const uint32_t bytes = e.blob_len;
    const uint32_t off = atomicAdd(&T.cnt[PVT_CARRY], bytes);
    if ((uint64_t)off + bytes > T.carry_cap) { atomicOr(&T.cnt[PVT_FLAGS], (uint32_t)PVT_F_CARRY); return; }
    const uint32_t *src = reinterpret_cast<const uint32_t *>(T.carry_in + e.blob);
    uint32_t *dst = reinterpret_cast<uint32_t *>(T.carry_out + off);
    for (uint32_t k = 0; k < bytes / 4; k++) dst[k] = src[k];
    e.blob = off;
    T.clist_out[atomicAdd(&T.cnt[PVT_NCARRY], 1u)] = fi;
}

// Stable LSD radix sort of the segment keys (rocPRIM onesweep)
extern "C" hipError_t pv_tcp_sort(void *tmp, size_t *tmp_bytes, uint64_t *kin, uint64_t *kout, uint32_t *vin,
                                  uint32_t *vout, size_t n, hipStream_t s)
{
    return rocprim::radix_sort_pairs(tmp, *tmp_bytes, kin, kout, vin, vout, n, 0, 64, s);
}
