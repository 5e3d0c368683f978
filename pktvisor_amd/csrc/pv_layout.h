// SPDX-License-Identifier: MPL-2.0
// pv_layout.h — device-state layout shared by the HIP kernels and the host runtime.
//
// A bucket (a 60 s period, AbstractMetricsManager.h:276-308) belongs to one handler. The
// Net and DNS managers shift independently (each on the first of *its own* events at or
// after its next_shift, :318-333), so each handler has its own window of bucket slots.
// Slot ids are the handler's period ordinal mod PV_SLOTS (deterministic, so every rank of a
// sharded run holds a period in the same slot). Physical slot s stores the Net bucket of
// Net slot s and the DNS bucket of DNS slot s side by side, in disjoint parts:
//   SUM region   uint64  [net part: net counters | payload-size histogram]
//                        [dns part: dns counters | udp-port / qtype / rcode tables]  (all-reduce SUM)
//   MIN region   int64   CPC first-occurrence global record index per coupon
//                        [net part: src, dst][dns part: qname]                      (all-reduce MIN)
//   top-N tables open addressing (key u64, count u64, aux u32) + name arena: table s
//                holds the Net metrics of Net slot s, table PV_SLOTS + s the DNS metrics
//                of DNS slot s (pv_tslot)
#pragma once
#include <stdint.h>

#define PV_SLOTS 16  // per handler: num_periods (<= 10) live + PV_MAX_SHIFTS new in one batch
#define PV_TABLES (2 * PV_SLOTS)
#ifndef PV_DNS_WAVES
#define PV_DNS_WAVES 8 // DNS pass: waves per workgroup (one resident workgroup per CU at its register count)
#endif
#define PV_MAX_SHIFTS 6 // period shifts per handler inside one device batch (the host splits longer batches)
#define PV_MAX_SUBNETS 16
// name arena partitions per slot: workgroup b allocates from partition b % PV_ARENA_PARTS,
// so no bump pointer is shared by more than a few workgroups
#define PV_ARENA_PARTS 64
// per-workgroup top-N update log (and its region-sorted copy, which also holds the dense
// IP entries): at most 7 top-N updates per record, plus one
// LDS cache flush (<= PV_CACHE_MAX entries) per bucket slot the workgroup touches
#define PV_MQ_PER_REC 7
#define PV_CACHE_MAX 4096

// group bits (same values as pv_net_group / pv_dns_group / pv_net2_group in include/pvgpu.h)
#define PV_N2G_COUNTERS 1u
#define PV_N2G_CARDINALITY 2u
#define PV_N2G_QUANTILES 4u
#define PV_N2G_TOP_GEO 8u
#define PV_N2G_TOP_IPS 16u
#define PV_N2G_ON 0x40000000u
#define PV_D2G_CARDINALITY (1u << 0)
#define PV_D2G_COUNTERS (1u << 1)
#define PV_D2G_QUANTILES (1u << 2)
#define PV_D2G_TOP_ECS (1u << 3)
#define PV_D2G_TOP_QTYPES (1u << 4)
#define PV_D2G_TOP_RCODES (1u << 5)
#define PV_D2G_TOP_SIZE (1u << 6)
#define PV_D2G_TOP_QNAMES (1u << 7)
#define PV_D2G_TOP_PORTS (1u << 8)
#define PV_D2G_XACT_TIMES (1u << 9)
#define PV_NET_COUNTERS_BIT 1u
#define PV_NET_CARDINALITY_BIT 2u
#define PV_NET_TOP_IPS_BIT 8u
#define PV_DNS_CARDINALITY_BIT (1u << 0)
#define PV_DNS_COUNTERS_BIT (1u << 1)
#define PV_DNS_QUANTILES_BIT (1u << 2)
#define PV_DNS_HISTOGRAMS_BIT (1u << 3)
#define PV_DNS_TOP_ECS_BIT (1u << 5)
#define PV_DNS_TRANSACTIONS_BIT (1u << 4)
#define PV_DNS_TOP_QNAMES_BIT (1u << 6)
#define PV_DNS_TOP_QNAMES_DETAILS_BIT (1u << 7)
#define PV_DNS_TOP_PORTS_BIT (1u << 8)

// ---- SUM region (uint64 words), per slot
#define PV_NET_CTRS 32
#define PV_DNS_CTRS 32
#define PV_PAYLOAD_BINS 65536
#define PV_PORT_BINS 65536
#define PV_QTYPE_BINS 65536
#define PV_RCODE_BINS 16
#define PV_OFF_NET 0
#define PV_OFF_PAYLOAD (PV_OFF_NET + PV_NET_CTRS)
// Net v2 (src/handlers/net/v2): its counters, then one payload-size histogram per direction
#define PV_NET2_CTRS 32
#define PV_OFF_NET2 (PV_OFF_PAYLOAD + PV_PAYLOAD_BINS)
#define PV_OFF_PAYLOAD2 (PV_OFF_NET2 + PV_NET2_CTRS) // + dir * PV_PAYLOAD_BINS
#define PV_SUM_NET_WORDS (PV_OFF_PAYLOAD2 + 3 * PV_PAYLOAD_BINS) // net part [0, PV_SUM_NET_WORDS)
#define PV_OFF_DNS PV_SUM_NET_WORDS
#define PV_OFF_PORT (PV_OFF_DNS + PV_DNS_CTRS)
#define PV_OFF_QTYPE (PV_OFF_PORT + PV_PORT_BINS)
#define PV_OFF_RCODE (PV_OFF_QTYPE + PV_QTYPE_BINS)
// DNS v2 (src/handlers/dns/v2), in place of v1 when configured: per transaction direction
// (0 in, 1 out, 2 unknown) its counters, then its port / qtype / rcode tables
#define PV_DNS2_CTRS 24
#define PV_OFF_DNS2 (PV_OFF_RCODE + PV_RCODE_BINS)              // + dir * PV_DNS2_CTRS
#define PV_OFF_PORT2 (PV_OFF_DNS2 + 4 * PV_DNS2_CTRS)           // + dir * PV_PORT_BINS
#define PV_OFF_QTYPE2 (PV_OFF_PORT2 + 3 * PV_PORT_BINS)         // + dir * PV_QTYPE_BINS
#define PV_OFF_RCODE2 (PV_OFF_QTYPE2 + 3 * PV_QTYPE_BINS)       // + dir * PV_RCODE_BINS
#define PV_SUM_WORDS (PV_OFF_RCODE2 + 4 * PV_RCODE_BINS)        // dns part [PV_OFF_DNS, PV_SUM_WORDS)

// net counters (src/handlers/net/v1/NetStreamHandler.h:69-96 + base event counters)
enum {
    NC_EVENTS = 0, NC_SAMPLES, NC_UDP, NC_TCP, NC_OTHER, NC_V4, NC_V6, NC_SYN, NC_IN, NC_OUT, NC_UNK, NC_TOTAL,
    NC_FILTERED, NC_COUNT
};
// DNS v2 counters per direction (src/handlers/dns/v2/DnsStreamHandler.h:75-120); D2_SEEN counts
// the responses and purge time-outs that set the direction up (DnsMetricsBucket::dir_setup)
enum {
    D2_SEEN = 0, D2_XACTS, D2_UDP, D2_TCP, D2_V4, D2_V6, D2_NX, D2_REFUSED, D2_SRVFAIL, D2_NOERROR, D2_NODATA, D2_AA,
    D2_AD, D2_CD, D2_TIMEOUT, D2_ORPHAN, D2_ECS,
    D2_DOT, D2_DOH, D2_CRYPT_UDP, D2_CRYPT_TCP, D2_DOQ, // dnstap socket protocols (Protocol, dns/v2 ...h:62-73)
    D2_N
};
// Net v2 counters (src/handlers/net/v2/NetStreamHandler.h:61-96): base events, then per
// direction d (0 in, 1 out, 2 unknown) at N2_DIR + 8 d
enum { N2_EVENTS = 0, N2_SAMPLES = 1, N2_FILTERED = 2, N2_DIR = 8 };
enum { N2_TOTAL = 0, N2_V4, N2_V6, N2_UDP, N2_TCP, N2_OTHER, N2_SYN };
// dns counters (src/handlers/dns/v1/DnsStreamHandler.h:94-139 + base event counters)
enum {
    DC_EVENTS = 0, DC_SAMPLES, DC_QUERIES, DC_REPLIES, DC_TCP, DC_UDP, DC_V4, DC_V6, DC_NX, DC_REFUSED, DC_SRVFAIL,
    DC_NOERROR, DC_NODATA, DC_TOTAL, DC_FILTERED, DC_XTOTAL, DC_XIN, DC_XOUT, DC_XTIMEOUT, DC_QECS, DC_COUNT
};

// ---- MIN region (int64 global record index), per slot: CPC lg_k = 11 => 2048 rows x 64 cols
#define PV_CPC_COUPONS (2048 * 64)
// v1 src_ips_in / dst_ips_out, v2 ips per direction (in, out, unknown), then the DNS qname
enum { CPC_SRC = 0, CPC_DST = 1, CPC_V2 = 2, CPC_QNAME = 5, CPC_QNAME2 = 6, CPC_SKETCHES = 9 }; // CPC_QNAME2 + dir: DNS v2
#define PV_MIN_WORDS (CPC_SKETCHES * PV_CPC_COUPONS)
#define PV_MIN_NET_WORDS (CPC_QNAME * PV_CPC_COUPONS) // net part [0, 5 * coupons), dns part after
#define PV_CPC_EMPTY 0x7fffffffffffffffLL

// ---- top-N metrics: key = metric << 56 | payload (56 bits)
enum {
    TM_NONE = 0, TM_IPV4 = 1, TM_IPV6 = 2, TM_QNAME2 = 3, TM_QNAME3 = 4, TM_NX = 5, TM_REFUSED = 6, TM_SRVFAIL = 7,
    TM_NODATA = 8, TM_NOERROR = 9, TM_SIZED = 10, TM_SLOW_IN = 11, TM_SLOW_OUT = 12,
    // dense metrics share the block cache, flushed into the SUM region
    TM_DENSE_PORT = 13, TM_DENSE_QTYPE = 14, TM_DENSE_RCODE = 15,
    // inserted straight into the global table (never through the block cache or update log,
    // whose keys carry 4-bit metric ids)
    TM_ECS = 16 // EDNS Client Subnet of a query (name record: family byte + 16 address bytes)
};
#define PV_KEY(metric, payload) (((uint64_t)(metric) << 56) | ((uint64_t)(payload) & 0x00ffffffffffffffULL))
// Net v2 top IPs share the Net table with v1's, told apart by a payload bit and carrying
// the direction: IPv4 payload 1 << 40 | dir << 34 | address, IPv6 1 << 55 | dir << 53 |
// 53-bit address hash
#define PV_V2_IP4(dir, ip) PV_KEY(TM_IPV4, (1ull << 40) | ((uint64_t)(dir) << 34) | (uint32_t)(ip))
#define PV_V2_IP6(dir, h) PV_KEY(TM_IPV6, (1ull << 55) | ((uint64_t)(dir) << 53) | ((h) & ((1ull << 53) - 1)))
#define PV_IS_V2_IP4(k) ((((k) >> 56) == TM_IPV4) && (((k) >> 40) & 1))
#define PV_IS_V2_IP6(k) ((((k) >> 56) == TM_IPV6) && (((k) >> 55) & 1))
// DNS v2 name keys: 1 << 55 | dir << 53 | 53-bit name fingerprint (v1 and v2 DNS never share a table)
#define PV_V2_DKEY(metric, dir, fp) PV_KEY(metric, (1ull << 55) | ((uint64_t)(dir) << 53) | ((fp) & ((1ull << 53) - 1)))
#define PV_IS_V2_DKEY(k) ((((k) >> 56) >= TM_QNAME2) && (((k) >> 55) & 1))
#define PV_KEY_METRIC(k) ((uint32_t)((k) >> 56))
// table of a (handler slot, metric): Net metrics (IPv4 / IPv6) in table slot, the DNS
// metrics in table PV_SLOTS + slot
#define PV_TSLOT(slot, metric) ((uint32_t)(slot) + (((metric) == TM_IPV4 || (metric) == TM_IPV6) ? 0u : (uint32_t)PV_SLOTS))

// Each slot's table is cut into regions of 2^PV_REGION_LOG2 entries (fewer when the table
// is smaller). A key lives in region (hash >> 40) & (regions - 1), at hash & (region - 1)
// plus linear probing that wraps inside the region, so one workgroup of pv_topn_merge
// can own a region outright and merge a batch's updates into it in LDS.
#define PV_REGION_LOG2 12
#ifndef PV_CB_THREADS
#define PV_CB_THREADS 1024 // pv_topn_combine workgroup size (the host launches the kernel's own bound)
#endif
#define PV_MAX_GRID 1024   // Net/DNS-pass workgroups per batch (pv_topn_merge's run table)
#define PV_MAX_REGIONS_LOG2 12 // table_log2 <= PV_REGION_LOG2 + PV_MAX_REGIONS_LOG2
#define PV_PROBES 256
// entry of the new-name list (pv_topn_merge -> pv_topn_names)
struct PvNewName {
    uint32_t slot; // table (PV_TSLOT)
    uint32_t rep;  // record index in the batch the name is decoded from
    uint64_t pos;  // table index (slot-relative offset included)
};

// aux word of a top-N entry: arena offset + 1 of its name record (0 = none)
// arena record: uint16 length, then bytes

// ---- flags word bits (device -> host)
enum {
    PVF_TABLE_FULL = 1u << 0,
    PVF_ARENA_FULL = 1u << 1,
    PVF_EVENTS_FULL = 1u << 2,
    PVF_VALUES_FULL = 1u << 3,
    PVF_BIG_CAPLEN = 1u << 4,
    PVF_NAMES_PENDING = 1u << 5 // created entries past the new-name list: aux = PV_AUX_PENDING | record
};
#define PV_AUX_PENDING 0x80000000u // (arena offsets stay below 2^31: arena_cap per table)

// DNS transaction event, one per DNS wire packet (for the pairing pass)
struct PvXEvent {
    uint64_t key;   // flowkey << 16 | txid
    uint32_t idx;   // record index within the batch
    uint32_t len;   // DNS message length (DnsLayer::getDataLen)
    int64_t sec;
    int32_t nsec;
    uint8_t qr;     // 1 = response
    uint8_t dir;    // PacketDirection: 0 toHost, 1 fromHost, 2 unknown
    uint8_t period; // DNS period index within the batch
    uint8_t pad;
};

// one transaction-derived value (quantile input), grouped per slot/kind on the host
enum { XV_FROM_US = 0, XV_TO_US = 1, XV_RATIO = 2, XV2_TIME = 3, XV2_RATIO = 6 }; // XV2_* + dir: DNS v2
struct PvXValue {
    uint64_t bits; // uint64 microseconds, or the IEEE-754 bits of the double ratio
    uint32_t slot; // slot | generation << 8
    uint32_t kind;
};

// radix selection over the device value buffer (pv_xv_hist): the selected kinds' prefixes so far
#define PV_XV_SEL 5 // XV_FROM_US, XV_TO_US, XV2_TIME + 0..2
struct PvXvSel {
    uint64_t prefix[PV_XV_SEL];
};

// a valid transaction whose period's slow threshold is not known yet
struct PvXValid {
    uint32_t idx; // response record index within the batch (PV_TCP_IDX: a TCP message record)
    uint8_t period, dir, pad0, pad1;
    uint64_t us;
};

// ---- DNS over TCP (PcapPlusPlus TcpReassembly + DnsTcpSessionData, device-resident)
// A DNS message cut from a reassembled TCP stream becomes a "message record" in the
// batch's TCP message arena: a classic-pcap record holding a raw-IPv4 (linktype 101)
// frame, IPv4 header (total length 0: no trim) + UDP header + the message, so every
// kernel that re-derives a name from a record (pv_topn_names, write_name, slow_check)
// reads it unchanged. Its index in the arena's offset list carries PV_TCP_IDX in events.
#define PV_TCP_IDX 0x80000000u
#define PV_TCP_REC_HDR 44u          // pcap record header 16 + IPv4 20 + UDP 8
#define PV_TCP_MIN_MSG 17u          // DnsTcpSessionData MIN_DNS_QUERY_SIZE
#define PV_TCP_MAX_OOO 50u          // TcpReassemblyConfiguration maxOutOfOrderFragments (PcapInputStream.cpp:79)
#define PV_TCP_TIMEOUT 30u          // PcapInputStream::TCP_TIMEOUT (PcapInputStream.h:97)
#define PV_TCP_RECLAIM 300u         // seconds after which a closed / timed-out flow entry is reused

// One TCP packet of a DNS-port flow that TcpReassembly does not drop at once (payload, or
// SYN / FIN / RST), emitted by the Net pass or, for a batch that may shift DNS windows,
// by pv_dns_prescan.
struct PvTcpSeg {
    uint32_t idx;        // record index in the batch
    uint32_t poff;       // absolute offset of the TCP payload in the record blob
    uint32_t seq;        // sequence number
    uint32_t fkey;       // hash5Tuple
    uint32_t sec, usec;  // packet timestamp at ConnectionData's timeval precision
    uint64_t ep;         // side: hash of (first IP layer's source address, source port)
    uint16_t plen, sport, dport;
    uint8_t flags;       // PV_TF_*
    uint8_t dirv6;       // PacketDirection | (first IP layer is IPv6) << 2
    uint32_t pad[2];
};
// PV_TF_NODATA: a TCP packet reassembly ignores (no payload and no SYN/FIN/RST, or no valid TCP
// header), emitted in the exact LRU mode for the cleanup that follows every TCP packet;
// PV_TF_CLOSE: a close-only segment the host's LRU replay adds for a connection it closes in a
// batch that holds none of its packets;
// PV_TF_EOC (with PV_TF_CLOSE): the end of the capture for an open connection, after the batch's
// last record (TcpReassembly::closeAllConnections, PcapInputStream.cpp:244,522; pv_tcp_eoc)
enum { PV_TF_FIN = 1, PV_TF_SYN = 2, PV_TF_RST = 4, PV_TF_EOC = 0x20, PV_TF_NODATA = 0x40, PV_TF_CLOSE = 0x80 };
static_assert(sizeof(PvTcpSeg) == 48, "three 16-B stores");

// TcpReassemblyData + DnsStreamHandler's TcpFlowData of one connection, carried across batches
struct PvTcpFlow {
    uint64_t tag;        // 0 empty, else 1 << 32 | flowKey
    uint32_t stage;      // TCP stage ordinal that last touched the entry
    uint8_t closed, tracked, v6, nsides;
    int8_t prev;         // prevSide
    uint8_t fin[2];
    uint8_t live;        // the connection exists (its first packet was seen)
    uint16_t sport, dport, port, pad1; // connData ports, metric port
    uint64_t ep[2];      // sides
    uint32_t seq[2];     // expected sequence per side
    uint32_t end_sec, end_usec; // ConnectionData::endTime (0 until a second packet)
    uint32_t lru_sec;    // time of the last LRU put (connection start / message ready)
    uint32_t close_sec;
    // DnsTcpSessionData per side: length bytes seen (0..2), message size, bytes held
    uint8_t inval[2], lenb[2];
    uint16_t size[2];
    uint32_t got[2];
    // carried bytes (carry arena): per side the held message bytes, then per side the
    // out-of-order fragments as {seq u32, len u32, bytes padded to 4}
    uint32_t blob, blob_len;
    uint16_t nfrag[2];
    uint32_t pad2[3];
};
static_assert(sizeof(PvTcpFlow) == 112, "flow entry size");
#define PV_TCP_FRAG_NIL 0xffffffffu
struct PvTcpFrag {
    uint64_t src;  // device address of the bytes
    uint32_t seq, len;
    uint32_t next, pad;
};



// Device pointers carry the global address space in the device compile, so the kernels
// emit global_* (not flat_*) memory instructions: flat accesses also count against
// lgkmcnt, which would make every LDS wait drain the in-flight HBM prefetch.
#if defined(__HIP_DEVICE_COMPILE__)
#define PV_G __attribute__((address_space(1)))
#else
#define PV_G
#endif

struct PvSubnets {
    uint32_t n4, n6;
    uint32_t v4_addr[PV_MAX_SUBNETS]; // in_addr.s_addr (network byte order as loaded LE)
    uint32_t v4_mask[PV_MAX_SUBNETS]; // htobe32(0xffffffff << (32 - cidr)); cidr 0 => match-all flag below
    uint32_t v4_all[PV_MAX_SUBNETS];
    uint8_t v6_addr[PV_MAX_SUBNETS][16];
    uint32_t v6_cidr[PV_MAX_SUBNETS];
};

// DNS filter bits (PvParams::f_flags)
#define PV_MAX_QTYPES 16
#define PV_MAX_QNAMES 8
#define PV_MAX_SUFFIXES 4
enum { PVDF_EXCLUDE_NOERROR = 1, PVDF_ONLY_RCODE = 2, PVDF_ANSWER_COUNT = 4, PVDF_ONLY_QUERIES = 8, PVDF_ONLY_RESPONSES = 16,
       PVDF_ONLY_QTYPE = 32, PVDF_ONLY_QNAME = 64, PVDF_ONLY_QSUFFIX = 128,
       PVDF_ONLY_DNSSEC = 256, PVDF_FILTER_ALL = 512, PVDF_PSL = 1024,
       // DNS v2 filters (dns/v2/DnsStreamHandler.cpp:61-170,484-609): PVDF_V2 selects their semantics
       // (responses: rcode / answer_count / DNSSEC / qtype, queries: qname / suffix, both: the
       // transaction directions; filtered messages stay transaction events)
       PVDF_V2 = 2048, PVDF2_NOIN = 4096, PVDF2_NOOUT = 8192, PVDF2_NOUNK = 16384, PVDF2_RCODE = 32768,
       PVDF2_QNAME = 65536 };
// public_suffix_list table on the device (pv_host.cpp psl_blob): 512 slots of {FNV-1a of the
// last label, byte offset, length, first suffix | count << 16}, then per suffix {offset, length}
#define PV_PSL_SLOTS 512
#define PV_PSL_SFX_WORD (PV_PSL_SLOTS * 4)
// One dnstap event for pv_dnstap_kernel (DnstapInputStream -> process_dnstap_cb of the Net
// and DNS handlers): the fields both handlers read, and the record (linktype 101: IPv4 or IPv6
// header with the query / response addresses, UDP header, the DNS message) write_name parses.
enum { PV_DT_EVENT_ONLY = 0, PV_DT_SIDE = 1, PV_DT_MESSAGE = 2 };
struct PvDtEv {
    uint32_t rec;      // record offset in the event arena
    uint32_t moff;     // absolute offset of the DNS message
    uint32_t mlen;     // DNS message bytes (PV_DT_MESSAGE)
    uint32_t size;     // protobuf frame length (the Net handler's payload size)
    uint32_t sec, nsec;
    uint16_t qport;
    uint8_t dir;       // Net: 0 toHost, 1 fromHost, 2 unknown (by message type)
    uint8_t l3;        // 0 unknown, 4, 6 (socket_family)
    uint8_t l4;        // 17, 6, 0 other (socket_protocol)
    uint8_t dns_mode;  // PV_DT_*
    uint8_t side;      // 0 query, 1 response (by message type)
    uint8_t filtered;  // dnstap_msg_type filter
    uint8_t qlen, rlen; // query / response address bytes (4, 16, else unusable)
    uint8_t pad[2];
    uint8_t qaddr[16], raddr[16];
    uint8_t pad2[12];
};
static_assert(sizeof(PvDtEv) == 80, "PvDtEv is five 16-B words");

// an update a full top-N region could not take inside a batch: kept for the retry after the
// table's purge (pv_topn_retry), so a burst of distinct keys degrades like the sketch's purge
// multi-GPU top-N exchange: the live tables and this rank's place (pv_topn_x*)
struct PvXTabs {
    uint32_t n, W, me, pad;
    uint32_t tb[PV_TABLES];
};

struct PvOvf {
    uint64_t key;
    uint32_t w, rep, slot, pad;
};

struct PvParams {
    const PV_G uint8_t *recs;
    const PV_G uint32_t *offs;
    uint64_t n;
    uint32_t linktype;
    uint32_t ts_nano;
    uint32_t net_groups, dns_groups;
    uint32_t net_filter_all; // every packet a filtered Net event (NetStreamHandler::_filtering without a geo database)
    // Net periods inside this batch: period p (0..n_shift) covers records [pstart[p-1], pstart[p])
    // (ts_sec in [thresh[p-1], thresh[p])); Net slot of each
    uint32_t n_shift;
    int64_t thresh[PV_MAX_SHIFTS];
    uint32_t slot_of[PV_MAX_SHIFTS + 1];
    uint32_t skip_before; // periods < skip_before are outside the kept window (no bucket updates)
    uint64_t pstart[PV_MAX_SHIFTS]; // first record index (in this batch) of period p+1
    // DNS periods (the DNS manager's own shifts): a DNS event with ts_sec in
    // [dthresh[p-1], dthresh[p]) is in DNS period p, kept iff p >= dskip_before
    uint32_t n_dshift;
    int64_t dthresh[PV_MAX_SHIFTS];
    uint32_t dslot_of[PV_MAX_SHIFTS + 1];
    uint32_t dskip_before;
    uint64_t gbase;
    PvSubnets nets;
    // device state
    PV_G uint64_t *sum;    // PV_SLOTS x PV_SUM_WORDS
    PV_G int64_t *cpc;     // PV_SLOTS x PV_MIN_WORDS
    PV_G uint64_t *tkeys;  // PV_TABLES x tcap
    PV_G uint64_t *tcnt;
    PV_G uint32_t *taux;
    uint32_t tcap_log2;
    PV_G uint8_t *arena;      // PV_TABLES x arena_cap, each table's split in PV_ARENA_PARTS partitions
    PV_G uint64_t *arena_top; // PV_TABLES x PV_ARENA_PARTS bump pointers (bytes used in the partition)
    uint64_t arena_cap;  // bytes per table
    PV_G uint64_t *dbits;      // pv_dns_prescan: one bit per record, set for a DNS event (after predicates)
    PV_G uint64_t *fbits;      // deep sampling with DNS filters: one bit per record (pv_dns_prescan) or per
                               // TCP message (pv_dns_tcp_filter), set for an event _filtering rejects
    PV_G PvXEvent *events;     // per-workgroup regions, indexed by workgroup tile range
    PV_G uint64_t *eecs;       // DNS v2 top_ecs: the ECS address of a query event (pad bits 3-4: family)
    PV_G uint64_t *ekeys;      // sort key per event slot: xact_sort_key (24-bit hash of (flow,txid) << 32 | rank)
    PV_G uint32_t *blk_events; // events appended by each workgroup
    PV_G uint64_t *skeys;      // packed keys (sort input)
    PV_G uint32_t *svals;      // packed event slot positions (sort input)
    PV_G uint32_t *n_events;   // [0] events of the batch, [1] responses
    PV_G uint32_t *n_keys;     // length of the batch's key list skeys / svals (events + sentinel slots)
    uint32_t want_events;
    uint32_t ekey_base;        // sort rank of the batch's first record (open queries carried in have rank 0)
    uint32_t wt_per_block; // 64-record wave tiles per workgroup (contiguous record range)
    uint64_t rec_bytes; // bytes of the record run (end of the last record)
    PV_G uint64_t *mq;    // per-workgroup top-N update logs: mq_cap x {key | slot << 60, w | rep << 32}
    PV_G uint32_t *mq_cnt; // entries per workgroup log
    PV_G uint64_t *stamps; // diagnostic builds (-DPV_STAMPS): 8 phase cycle sums per wave
    uint32_t mq_cap;
    uint32_t grid_main;   // workgroups of pv_net_kernel / pv_dns_kernel
    PV_G uint64_t *dq;    // per-workgroup DNS work lists (32-B DnsMsg), region = wt_per_block * 64
    PV_G uint32_t *dq_cnt;
    PV_G uint32_t *n_dns; // DNS messages found by the Net pass (status word)
    // top-N merge: regions per slot table (log2), the run table and the new-name list
    uint32_t reg_log2;
    PV_G uint32_t *tp_hands; // status word: bit h set when handler h (0 Net, 1 DNS) has top-N entries
    PV_G uint64_t *cb_run;  // [run key][XCD][combine workgroup / 8]: the workgroup's run of that
                            // run key in its sorted list (start | count << 24 | tables << 48)
    PV_G uint32_t *tab_live; // per table: entries held (bounded by pv_topn_purge)
    PV_G PvOvf *ovf;          // top-N updates a full region could not take (pv_topn_retry after a purge)
    PV_G uint32_t *ovf_cnt;   // [0] entries, [1] tables they belong to (bit mask)
    uint32_t ovf_cap;
    uint32_t net2_groups;   // Net v2 handler attached: PV_N2G_* group bits | PV_N2G_ON (0 = not attached)
    uint32_t dns2_groups;   // DNS v2 in place of v1: PV_D2G_* group bits | PV_N2G_ON (0 = DNS v1)
    PV_G uint64_t *tp_buf; // pv_topn_combine: entries its LDS table could not take (spill)
    PV_G uint32_t *nn_cnt;
    PV_G PvNewName *nn;
    uint32_t nn_cap;
    PV_G uint64_t *iplog; // dense IP log: one entry per record of the batch (Net pass)
    // compact IP log of the register-window Net pass (ip_compact): the IPv4 address of each
    // record (0: no entry), its direction bit per 64-record tile, and per grid workgroup range
    // the other entries (IPv6 keys of general-path records) in iplog at the range's base
    PV_G uint32_t *iplog32;
    PV_G uint64_t *ipdir;
    PV_G uint32_t *ipx_cnt;
    PV_G uint32_t *ipx_rep; // the exception entries' record indices (names of IPv6 keys)
    uint64_t ip_base;     // slot << 60 | TM_IPV4 << 56 | cardinality << 33: the entries' common bits
    uint32_t ip_compact;
    // span Net pass (pv_net_kernel_span): the records the fast path does not take, deferred to
    // pv_net_slow_list (record indices at each range's base, each range's count)
    PV_G uint32_t *slow_list;
    PV_G uint32_t *slow_cnt;
    PV_G uint32_t *n_slow; // deferred records of the batch (status word; pv_net_slow_list exits at 0)
    // top_ecs of the UDP DNS pass: {key lo, key hi, slot, record} per query with an ECS option,
    // inserted into the global table by pv_dns_ecs after the pass (no device call in the pass)
    PV_G uint32_t *ecs_list; // four words an entry
    PV_G uint32_t *n_ecs; // status word
    uint32_t ecs_cap;
    PV_G uint64_t *trash; // 64-B line per Net-pass wave for stores that have nothing to store
    PV_G uint64_t *cb;    // combined update lists sorted by table region, mq_cap entries per workgroup
    PV_G uint32_t *cb_cnt;
    PV_G uint32_t *cb_hm; // per combine workgroup: handlers with entries (bit 0 Net, 1 DNS); run words of the others unwritten
    uint32_t cb_fan;      // grid ranges per combine workgroup (its list: cb_fan x mq_cap entries)
    uint32_t cb_grid;     // combine workgroups: ceil(grid_main / cb_fan)
    uint32_t xmerge;      // pv_topn_merge over received multi-GPU entries (64-bit weights, no names)
    uint32_t x_lo, x_hi;  // its regions [x_lo, x_hi)
    uint32_t dbg; // profiling knob (PV_DEBUG_STAGES env): 1 stop after staging, 2 after parse, 4 no DNS lane,
                  // 16 no DNS name decode, 32 no DNS table updates
    PV_G uint32_t *flags;
    // DNS v1 filters (DnsStreamHandler::_filtering, dns/v1/DnsStreamHandler.cpp:538-648)
    uint32_t f_flags, f_rcode_mask, f_ancount, f_nq;
    uint16_t f_qt[PV_MAX_QTYPES];
    uint32_t f_nqn;
    uint64_t f_qn[PV_MAX_QNAMES]; // only_qname: name fingerprints (fp56 of the lower-case name)
    uint32_t f_nsx;                    // only_qname_suffix: list length, then per suffix
    uint32_t f_sxl[PV_MAX_SUFFIXES];   // its length and
    uint64_t f_sxh[PV_MAX_SUFFIXES];   // its polynomial hash (ph_step over the lower-case chars)
    PV_G uint8_t *sfx_of;              // per record of the batch: the matched suffix size (DNS pass writes)
    // DNS over TCP. Emission (Net pass of a one-span batch, else pv_dns_prescan): segments of
    // DNS-port TCP flows, their payload bytes, and per 64-record tile the mask of TCP records
    uint32_t tcp_emit;
    uint32_t tseg_cap;
    PV_G PvTcpSeg *tseg;
    PV_G uint32_t *tseg_cnt;           // [0] segments [1] payload bytes
    PV_G uint64_t *tmask;
    // the TCP DNS pass (pv_dns_tcp): message records replace recs / offs (linktype 101), dq
    // holds the messages; a message's order in the batch is ord = record * 4 + sub
    uint32_t tcp_pass, tcp_nmsg;
    uint32_t ord_lo, ord_hi, ord_base; // this span's messages: ord in [ord_lo, ord_hi); ord_base = span start * 4
    uint32_t tap; // dnstap events (pv_dnstap_kernel): IPv6 top-N names take the address the key hashes
    // deep sampling (deep_sample_rate < 100, AbstractMetricsManager::new_event): bit i set =
    // record i's Net event / DNS event draws "not deep" (the managers' jsf32 draws, on the host)
    const PV_G uint32_t *ndeep_net, *ndeep_dns;
    uint32_t dpos[PV_MAX_SHIFTS];      // span-relative ord of the event that shifts DNS period k+1
    PV_G const uint32_t *psl;          // public_suffix_list table (PVDF_PSL)
};

// pv_fill_multi's segment list (kernel argument)
#define PV_FILL_SEGS 24
struct PvFillSeg {
    void *p;
    uint64_t n;
    uint64_t v;
    uint32_t w32; // 1: 32-bit words
    uint32_t pad;
};
struct PvFillList {
    PvFillSeg s[PV_FILL_SEGS];
    uint32_t n;
};

// A parameter block passed by value to pv_store_blob (kernel arguments): the per-batch upload
// without a copy command (a small host-to-device copy is a blit dispatch plus the stream's
// dependency on it)
#define PV_BLOB_WORDS 128 // 16-B words (2 KiB)
struct PvBlob {
    uint32_t w[4 * PV_BLOB_WORDS];
};

struct PvXactParams {
    PvParams P;            // record access + top-N tables (slow transaction names)
    const PV_G PvXEvent *events;
    const PV_G uint64_t *skeys; // sorted xact_sort_key (hash24(key) << 32 | rank)
    const PV_G uint32_t *svals; // event position for each sorted key
    uint32_t n;
    uint32_t ttl_s, ttl_ms;
    uint32_t quantiles; // bit 0: quantiles group (time and ratio values), bit 1: histograms (time values)
    uint32_t slot_gen[PV_MAX_SHIFTS + 1]; // DNS slot | generation << 8 per DNS period
    float thr_from[PV_MAX_SHIFTS + 1];    // p90 slow thresholds per period, < 0 = not known yet
    float thr_to[PV_MAX_SHIFTS + 1];
    PV_G PvXValue *vals;
    PV_G uint32_t *n_vals;
    uint32_t vals_cap;
    PV_G PvXValid *valid;
    PV_G uint32_t *n_valid;
    // DNS queries still open from earlier batches (TransactionManager's map carried across
    // batches): sorted-key values with PV_PEND_FLAG index the event store `pend` (a query-only
    // batch's own event regions become the store as they lie, so it may be sparse); pv_xact_carry
    // writes the queries still open after this batch densely to pend_out / pkeys_out /
    // pvals_out, counting n_pend_out
    const PV_G PvXEvent *pend;
    PV_G PvXEvent *pend_out;
    const PV_G uint64_t *pecs; // DNS v2 top_ecs: ECS addresses of the carried queries (pend), and of pend_out
    PV_G uint64_t *pecs_out;
    PV_G uint64_t *pkeys_out;
    PV_G uint32_t *pvals_out;
    PV_G uint32_t *n_pend_out;
    // shard-edge stubs: responses that are the first event of their (flow, txid) in this
    // context's whole stream ("orphans"; they may answer a query open at the end of the
    // previous shard), appended with pad = slot | kept << 7
    PV_G PvXEvent *orph;
    PV_G uint32_t *n_orph;
    uint32_t orph_cap;
    // DNS v2 stubs: the first-occurrence order of each (a response's qname CPC order when it
    // becomes an edge pair), next to orph; null in v1 runs
    PV_G int64_t *orph_ord;
    // TCP message records (events whose idx carries PV_TCP_IDX) and their suffix sizes
    // (public_suffix_list, DNS v2)
    const PV_G uint8_t *trecs;
    const PV_G uint32_t *toffs;
    const PV_G uint8_t *tsfx;
    // DNS v2: per period and direction the p90 slow threshold (< 0 = not known yet)
    float thr2[PV_MAX_SHIFTS + 1][3];
    // sharded runs (pv_set_slow_defer): queries with no earlier event of their key whose second
    // is below this horizon are appended to the stub list too (a query of an earlier shard still
    // open there is overwritten by them, TransactionManager::start_transaction); 0 = none
    int64_t edge_h;
};
#define PV_PEND_FLAG 0x80000000u
// A DNS v2 transaction across a shard edge (pv_edge_carry): a query an earlier shard left open
// and the response that is the first event of its key in this shard, accounted on the response
// (pv_xact_edge2). r.idx indexes the edge run's record blobs, r.period its period table.
struct PvEdgePair {
    PvXEvent q, r;
    uint64_t qaddr; // the query's ECS address (top_ecs)
    int64_t order;  // the response's first-occurrence order in the stream
    uint64_t us;    // transaction time
};

// TCP stage parameters (pv_tcp_* kernels)
struct PvTcpParams {
    const PV_G PvTcpSeg *seg;     // segments of the batch (emission order)
    const PV_G uint64_t *skey;    // sorted (fkey << 32 | record index)
    const PV_G uint32_t *sval;    // segment index per sorted key
    uint32_t n_seg;
    uint32_t stage;               // ordinal of this stage (>= 1)
    uint32_t now_sec;             // first record second of the batch (entry reclaim)
    uint32_t flow_cap_log2;
    PV_G PvTcpFlow *flows;
    PV_G uint32_t *run_flow;      // per sorted segment: flow entry of the run it starts (else ~0)
    // last-TCP-second structure: per 64-record tile the mask of TCP records, and the prefix
    // maximum (+1) of TCP record seconds over earlier tiles (carried over batches in lt_carry)
    const PV_G uint64_t *tmask;
    PV_G uint32_t *tpm;
    PV_G uint32_t *lt_carry;
    const PV_G uint8_t *recs;     // the batch's records (segment payloads, TCP record seconds)
    const PV_G uint32_t *offs;
    uint32_t n_tiles, ts_nano;
    // carried bytes: in (previous stage) and out (this stage), with the carried-flow lists
    const PV_G uint8_t *carry_in;
    PV_G uint8_t *carry_out;
    uint64_t carry_cap;
    const PV_G uint32_t *clist_in;
    uint32_t n_clist_in;
    PV_G uint32_t *clist_out;
    PV_G PvTcpFrag *frags;        // fragment node pool
    uint32_t frag_cap;
    // message output: arena of message records, their offsets and DnsMsg work items
    PV_G uint8_t *marena;
    uint64_t marena_cap;
    PV_G uint32_t *moffs;
    PV_G uint64_t *mq;            // 32-B DnsMsg items (same layout as the UDP work lists)
    uint32_t mq_cap;
    PV_G uint32_t *cnt;           // [0] messages [1] arena bytes [2] carry bytes [3] carried flows [4] frag nodes [5] flags
    // exact LRU mode (pv_set_tcp_exact_lru; tcp_packet_reassembly_cache_limit implies it): every
    // TCP packet is a segment, a dry run records the LRU events of every sorted segment (lru_ev:
    // flags | dir << 8, second, the LRU time of its last put: ConnectionData::endTime, 0 until
    // the connection's second packet) and leaves the flow table, the carried bytes and lt_carry
    // as they were; the host replays PcapInputStream's LRU list over them and the run after it
    // closes each flow the replay closed (fclose per segment index, read at the flow's first
    // sorted segment: record index after which it closes, that record's second and direction).
    // Outside it the device times a connection out by itself (lt_before).
    uint32_t dry, exact;
    PV_G uint32_t *lru_ev;
    const PV_G uint32_t *fclose;
};
enum { PVT_NMSG = 0, PVT_ARENA, PVT_CARRY, PVT_NCARRY, PVT_NFRAG, PVT_FLAGS, PVT_WORDS };
// LRU events of one segment (lru_ev flags): a connection start's put, a message delivery's put,
// the connection closed (FIN/RST) in it, closed by the 30 s timeout ahead of it; HOLD: after it
// the connection holds a fragment that closing it would deliver (the close's own put)
enum { PVT_EV_NEW = 1, PVT_EV_PUT = 2, PVT_EV_CLOSE = 4, PVT_EV_TIMEOUT = 8, PVT_EV_HOLD = 16 };
#define PVT_FCLOSE_NONE 0xffffffffu
enum { PVT_F_TABLE = 1, PVT_F_ARENA = 2, PVT_F_CARRY = 4, PVT_F_FRAGS = 8, PVT_F_MSGS = 16 };

// Device record index of an ingest chunk (pv_index.hip)
#define PV_IX_SEG 2048u
#define PV_IX_NONE 0xffffffffffffffffull
#define PV_IX_STOP (1ull << 63) // exit flag: the walk stopped at a truncated record / the end
struct PvIxParams {
    const PV_G uint8_t *recs;
    uint64_t bytes;
    uint32_t nseg, frac_lim, sec0, first; // first: offset of the first record (< PV_IX_SEG)
    PV_G uint64_t *start;      // per segment: first record start (PV_IX_NONE: none found)
    PV_G uint64_t *exit[2];    // per segment: position after its records (| PV_IX_STOP), double-buffered
    PV_G uint32_t *cnt;        // per segment: records starting in it
    PV_G uint32_t *base;       // per segment + 1: exclusive prefix of cnt
    PV_G uint32_t *offs;       // record offsets
    uint64_t max_records;
    PV_G uint32_t *status;     // [0] fix pass changed something, [1] sec changes, [2] non-monotone
    PV_G uint32_t *sci, *scs;  // sec change points (unordered; the host sorts them)
    uint32_t max_changes;
};

