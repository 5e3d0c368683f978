/* SPDX-License-Identifier: MPL-2.0
 *
 * pvgpu.h — C-ABI of the MI355X-native Net+DNS per-packet path.
 *
 * This is the drop-in boundary a pktvisor build binds to (see INTEGRATION.md for
 * the StreamHandler / InputStream shim). Plain pointers and sizes only; no
 * exceptions cross it; every call returns 0 on success or a negative pv_status,
 * and pv_last_error() returns the message of the last failure on a context.
 *
 * Mapping to the reference (/root/reference):
 *   pv_create / pv_destroy ........ NetStreamHandler / DnsStreamHandler ctor+start()/stop()
 *                                   (src/handlers/net/v1/NetStreamHandler.cpp:31-130,
 *                                    src/handlers/dns/v1/DnsStreamHandler.cpp:30-232) and
 *                                   the window config of AbstractMetricsManager
 *                                   (src/AbstractMetricsManager.h:351-389)
 *   pv_index_records .............. the record walk of PcapInputStream::_open_pcap
 *                                   (src/inputs/pcap/PcapInputStream.cpp:471-527)
 *   pv_process_host /
 *   pv_process_device ............. per-record dispatch PcapInputStream::process_raw_packet
 *                                   (PcapInputStream.cpp:380-428) into
 *                                   NetStreamHandler::process_packet_cb (net/v1 ...cpp:161-169)
 *                                   and DnsStreamHandler::process_udp_packet_cb
 *                                   (dns/v1 ...cpp:270-302), for a whole block of records
 *   pv_set_start_tstamp /
 *   pv_set_end_tstamp ............. start_tstamp_signal / end_tstamp_signal
 *                                   (PcapInputStream.cpp:494-500,514-517;
 *                                    AbstractMetricsManager.h:423-437)
 *   pv_window_json ................ StreamHandler::window_json(j, period, merged)
 *                                   (src/StreamHandler.h:71-77, AbstractMetricsManager.h:480-504,601-647)
 *   pv_window_prometheus .......... StreamHandler::window_prometheus(out, add_labels)
 *                                   (src/StreamHandler.h:71-77, AbstractMetricsManager.h:506-531;
 *                                    NetStreamHandler.cpp:332-388, DnsStreamHandler.cpp:1139-1238)
 *   pv_window_opentelemetry ....... StreamHandler::window_opentelemetry(scope, start, end, add_labels)
 *                                   (AbstractMetricsManager.h:533-575; Metrics.cpp:22-36,82-96)
 *   pv_add_static_label ........... Metric::add_static_label (src/Metrics.h, Metrics.cpp:129-155)
 *   pv_state_* / pv_reduce_* ...... the bucket merge (AbstractMetricsBucket::merge,
 *                                   AbstractMetricsManager.h:177-195) split into
 *                                   collective-friendly regions for a multi-GPU reduce
 */
#ifndef PVGPU_H
#define PVGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pv_ctx pv_ctx;

enum pv_status {
    PV_OK = 0,
    PV_EINVAL = -1,    /* bad argument / config (message in pv_last_error) */
    PV_EHIP = -2,      /* HIP runtime failure */
    PV_ECAPACITY = -3, /* a device table overflowed its configured capacity */
    PV_EUNSUPPORTED = -4,
    PV_ENODEV = -5     /* no HIP device / extension not usable */
};

/* Metric groups (names as the reference's _group_defs). */
enum pv_net_group { PV_NET_COUNTERS = 1u << 0, PV_NET_CARDINALITY = 1u << 1, PV_NET_TOP_GEO = 1u << 2, PV_NET_TOP_IPS = 1u << 3 };
enum pv_dns_group {
    PV_DNS_CARDINALITY = 1u << 0, PV_DNS_COUNTERS = 1u << 1, PV_DNS_QUANTILES = 1u << 2, PV_DNS_HISTOGRAMS = 1u << 3,
    PV_DNS_TRANSACTIONS = 1u << 4, PV_DNS_TOP_ECS = 1u << 5, PV_DNS_TOP_QNAMES = 1u << 6,
    PV_DNS_TOP_QNAMES_DETAILS = 1u << 7, PV_DNS_TOP_PORTS = 1u << 8
};
/* Net v2 handler groups (src/handlers/net/v2/NetStreamHandler.h:25-31, _group_defs :262-267). */
enum pv_net2_group {
    PV_NET2_COUNTERS = 1u << 0, PV_NET2_CARDINALITY = 1u << 1, PV_NET2_QUANTILES = 1u << 2, PV_NET2_TOP_GEO = 1u << 3,
    PV_NET2_TOP_IPS = 1u << 4
};
/* DNS v2 handler groups (src/handlers/dns/v2/DnsStreamHandler.h:40-52, _group_defs :565-575). */
enum pv_dns2_group {
    PV_DNS2_CARDINALITY = 1u << 0, PV_DNS2_COUNTERS = 1u << 1, PV_DNS2_QUANTILES = 1u << 2, PV_DNS2_TOP_ECS = 1u << 3,
    PV_DNS2_TOP_QTYPES = 1u << 4, PV_DNS2_TOP_RCODES = 1u << 5, PV_DNS2_TOP_SIZE = 1u << 6, PV_DNS2_TOP_QNAMES = 1u << 7,
    PV_DNS2_TOP_PORTS = 1u << 8, PV_DNS2_XACT_TIMES = 1u << 9
};
#define PV_DNS2_DEFAULT_GROUPS (PV_DNS2_CARDINALITY | PV_DNS2_COUNTERS | PV_DNS2_QUANTILES | PV_DNS2_TOP_QNAMES | \
                                PV_DNS2_TOP_RCODES | PV_DNS2_TOP_QTYPES)
#define PV_NET2_DEFAULT_GROUPS (PV_NET2_COUNTERS | PV_NET2_CARDINALITY | PV_NET2_QUANTILES | PV_NET2_TOP_GEO | PV_NET2_TOP_IPS)
/* OR'ed into pv_config.net_groups / dns_groups: the bits are the enabled set even when it is
 * empty ("disable: [all]"); without it 0 selects the handler's default groups */
#define PV_GROUPS_SET 0x80000000u
#define PV_NET_DEFAULT_GROUPS (PV_NET_COUNTERS | PV_NET_CARDINALITY | PV_NET_TOP_GEO | PV_NET_TOP_IPS)
#define PV_DNS_DEFAULT_GROUPS (PV_DNS_CARDINALITY | PV_DNS_COUNTERS | PV_DNS_QUANTILES | PV_DNS_TRANSACTIONS | \
                               PV_DNS_TOP_QNAMES | PV_DNS_TOP_PORTS)

typedef struct pv_config {
    const char *host_spec;   /* comma-separated CIDRs, PcapInputStream "host_spec" (may be NULL) */
    uint32_t num_periods;    /* window history 1..10 ("num_periods", default 5) */
    uint32_t topn_count;     /* "topn_count", default 10 */
    uint32_t xact_ttl_ms;    /* "xact_ttl_ms", default 5000 */
    uint32_t net_groups;     /* pv_net_group bits (| PV_GROUPS_SET); 0 => defaults */
    uint32_t dns_groups;     /* pv_dns_group bits (| PV_GROUPS_SET); 0 => defaults */
    uint32_t linktype;       /* pcap linktype of the records (1 = Ethernet) */
    uint32_t ts_nano;        /* 1 if record timestamps are ns (magic a1b23c4d) */
    int32_t device;          /* HIP device ordinal, -1 => current */
    uint32_t table_log2;     /* log2 slots of each per-period top-N table, 0 => 22 */
    uint64_t max_records;    /* largest batch that will be submitted (sizes scratch) */
    uint32_t topn_percentile_threshold; /* "topn_percentile_threshold" 0..99 (TopN::to_json, src/Metrics.h:510-521,577-590) */
    uint32_t net_filter_all; /* nonzero: every packet is a filtered Net event (geo / ASN filters without a geo
                                database, NetStreamHandler::_filtering, net/v1/NetStreamHandler.cpp:223-283) */
    uint32_t net2_groups;    /* Net v2 handler ("net", src/handlers/net/v2) attached next to v1: pv_net2_group bits
                                | PV_GROUPS_SET, or PV_NET2_ATTACH for its default groups; 0 = not attached */
    uint32_t dns2_groups;    /* DNS v2 handler ("dns", src/handlers/dns/v2) in place of v1: pv_dns2_group bits
                                | PV_GROUPS_SET, or PV_NET2_ATTACH for its default groups; 0 = DNS v1. Filters
                                (pv_set_dns_filters, v2 keys incl. only_xact_directions), top_ecs and the
                                multi-GPU edge replay (pv_edge_carry) are built; geo/ASN filters are refused */
    uint32_t deep_sample_rate; /* "deep_sample_rate" 1..100 (0 = 100): each manager draws jsf32() % 100 < rate
                                  per event (AbstractMetricsManager::new_event, src/AbstractMetricsManager.h:318-333);
                                  a non-deep event counts in the counters only. Every handler version, DNS
                                  filters and DNS over TCP sample; refused (PV_EUNSUPPORTED) only with the Net
                                  geo filters (net_filter_all: no geo database) */
} pv_config;
#define PV_NET2_ATTACH 0x40000000u

/* DNS v1 filters, the typed form of the "exclude_noerror", "only_rcode", "answer_count",
 * "only_queries", "only_responses" and "only_qtype" handler config keys
 * (DnsStreamHandler::start, src/handlers/dns/v1/DnsStreamHandler.cpp:60-150; applied as
 * _filtering :538-648). A filtered DNS packet is an event plus the `filtered` counter and
 * nothing else (process_filtered, :1341-1347). only_rcode is the input-proxy predicate
 * (:485-508): packets it rejects (queries, other rcodes) are not events at all.
 * geoloc / asn are not built (no geo database). only_qname is matched by the DNS
 * pass's 56-bit name fingerprint (the key its top-N tables use), only_qname_suffix by the
 * 64-bit polynomial hash of the name's last L characters. */
typedef struct pv_dns_filters {
    uint32_t exclude_noerror;   /* nonzero: filter rcode 0 (queries too); wins over only_rcode */
    uint32_t only_rcode_mask;   /* bit r: rcode r wanted (r <= 15, a known RCodeNames value) */
    int32_t answer_count;       /* ANCOUNT wanted, -1 = off */
    uint32_t only_queries;      /* nonzero: filter responses */
    uint32_t only_responses;    /* nonzero: filter queries */
    uint32_t n_qtypes;          /* entries used in qtypes (<= 16), 0 = off */
    uint16_t qtypes[16];        /* first-query qtype wanted (QTypeNames values) */
    uint32_t n_qnames;          /* "only_qname" entries (<= 8), 0 = off; input predicate like only_rcode */
    const char *const *qnames;  /* first-query names wanted (compared lower-case); not with only_rcode */
    uint32_t n_qname_suffixes;  /* "only_qname_suffix" entries (<= 4), 0 = off */
    const char *const *qname_suffixes; /* lower-cased; the first one the name ends with sets the
                                          aggregateDomain suffix size */
    uint32_t only_dnssec_response; /* nonzero: filter all but responses with an RRSIG answer */
    uint32_t filter_all;        /* nonzero: filter every DNS event that passes the predicates (geoloc_notfound /
                                   asn_notfound without a geo database, :619-642) */
    uint32_t public_suffix_list; /* nonzero: "public_suffix_list" config (DnsStreamHandler::_configs,
                                   :648-657): the first query's match_public_suffix size is the
                                   aggregateDomain suffix size for top_qname2/3; ignored with
                                   only_qname_suffix, as in the reference */
    uint32_t v2;                /* nonzero: the DNS v2 handler's filters (dns/v2/DnsStreamHandler.cpp:
                                   61-170,484-609): rcode (exclude_noerror / only_rcode), answer_count,
                                   DNSSEC and qtype test responses, qname and qname suffix test queries,
                                   no input predicate; a filtered message still opens / ends its
                                   transaction (process_filtered :1147-1174). only_queries /
                                   only_responses / public_suffix_list / filter_all are not v2 keys */
    uint32_t xact_dirs_disabled; /* v2 only_xact_directions: bit 0 in, 1 out, 2 unknown filtered */
} pv_dns_filters;

/* Replaces DnsStreamHandler::start's filter setup (dns/v1/DnsStreamHandler.cpp:60-150). Call
 * before the first batch; NULL clears. PV_EINVAL with the reference's ConfigException text
 * for an unknown rcode/qtype. */
int pv_set_dns_filters(pv_ctx *ctx, const pv_dns_filters *f);

/* PcapInputStream's "tcp_packet_reassembly_cache_limit" (src/inputs/pcap/PcapInputStream.cpp:97-99):
 * the capacity of the LRU list of TCP connections (254-283,449-465); a connection start or a
 * message delivery beyond it evicts the least recently used connection, which is closed
 * (closeConnection). 0 (the default): the reference's DEFAULT_LRULIST_SIZE behaviour without
 * the capacity check. A limit implies the exact LRU mode below. Call before the first batch. */
int pv_set_tcp_reassembly_limit(pv_ctx *ctx, uint64_t limit);
/* The exact LRU mode of DNS over TCP (on != 0): PcapInputStream's LRU list of every TCP
 * connection (PcapInputStream.cpp:254-283,429-465) is replayed on the host per batch from a dry
 * run of the device TCP stage: puts with the connection's endTime (0 until its second packet, so
 * a connection first seen with data, e.g. a capture that misses the handshake, leaves as soon as
 * it reaches the list's tail), after every TCP packet at most MAX_TCP_CLEANUPS (100) 30 s
 * time-outs, then the evictions; the device closes what the replay closes. Off (the default):
 * the device times each DNS-port connection out by itself 30 s after its last put's second,
 * which is the same outcome except for those zero-endTime connections and more than 100
 * time-outs at one packet. The exact mode costs a second run of the TCP stage and a host walk
 * over every TCP packet of a batch. Call before the first batch. */
int pv_set_tcp_exact_lru(pv_ctx *ctx, int on);
/* A classic-BPF instruction (struct sock_filter, linux/filter.h): what libpcap's pcap_compile
 * produces and `tcpdump -dd EXPR` prints. */
typedef struct pv_bpf_insn {
    uint16_t code;
    uint8_t jt, jf;
    uint32_t k;
} pv_bpf_insn;
/* The pcap input's "bpf" filter (PcapInputStream::_open_pcap: reader->setFilter(bpf),
 * src/inputs/pcap/PcapInputStream.cpp:485-488, pcap_offline_filter semantics): records the
 * program answers 0 for never reach the handlers (no event, no timestamp, no period shift).
 * Applies to pv_process_host input from the next call; the program comes compiled (libpcap is
 * not linked). n = 0 removes the filter. PV_EINVAL for a program the classic-BPF checker
 * refuses (unknown opcode, jump out of range, scratch index >= 16, division by a constant 0,
 * no final return). pv_process_host and pv_process_device input are both filtered on the device
 * (pv_bpf_keep: one lane per record runs the program; the kept records are compacted in HBM). */
int pv_set_bpf(pv_ctx *ctx, const pv_bpf_insn *prog, uint32_t n);
/* Pure host functions of the same machine: validate a program (PV_OK / PV_EINVAL); run it on one
 * frame (wirelen = the record's orig_len, buflen = its incl_len; 0 = drop); copy the records of
 * a block of classic-pcap records the program keeps to out (out may equal recs). */
int pv_bpf_validate(const pv_bpf_insn *prog, uint32_t n);
uint32_t pv_bpf_run(const pv_bpf_insn *prog, const uint8_t *frame, uint32_t wirelen, uint32_t buflen);
int pv_bpf_filter_records(const pv_bpf_insn *prog, uint32_t n, const uint8_t *recs, size_t bytes, uint8_t *out,
                          size_t *out_bytes, uint64_t *kept);
/* Name or decimal -> code for kind 0 = rcode (RCodeNumbers) or 1 = qtype (QTypeNumbers),
 * case-insensitive, libs/visor_dns/dns.h:31-265; PV_EINVAL if unknown. Pure host function. */
int pv_dns_code(int kind, const char *name, uint32_t *value);

/* Result of one host-side walk over a run of classic-pcap records. */
typedef struct pv_index_info {
    uint64_t n_records;      /* records indexed */
    uint64_t bytes_used;     /* bytes of whole records consumed */
    int64_t first_sec, first_nsec, last_sec, last_nsec;
    uint32_t monotone;       /* 1 if ts_sec never decreases inside the run */
    uint32_t n_sec_changes;  /* entries written to sec_change_* */
} pv_index_info;

const char *pv_version(void);
int pv_device_count(int *count);

int pv_create(const pv_config *cfg, pv_ctx **out);
void pv_destroy(pv_ctx *ctx);
const char *pv_last_error(const pv_ctx *ctx);

/* Walk records [recs, recs+bytes): per-record byte offsets (relative to recs)
 * into offsets[max_records], and the points where ts_sec changes into
 * sec_change_idx/sec_change_sec[max_changes] (index of the first record with
 * that second). Pure host function; no context needed. */
int pv_index_records(const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets, uint64_t max_records,
                     uint32_t *sec_change_idx, uint32_t *sec_change_sec, uint32_t max_changes, pv_index_info *info);

/* The same index computed on the device (pv_index.hip: segment guesses validated along the
 * true chain, then offsets and ts_sec change points), for a block of at most one ingest
 * chunk (64 MiB, PV_INGEST_CHUNK_MB); the outputs equal pv_index_records'. A block whose
 * guesses do not settle within 64 validation passes (payloads forged to look like record
 * chains across more than 64 segments) is walked on the host instead. */
int pv_index_records_device(pv_ctx *ctx, const uint8_t *recs, size_t bytes, uint32_t *offsets, uint64_t max_records,
                            uint32_t *sec_change_idx, uint32_t *sec_change_sec, uint32_t max_changes,
                            pv_index_info *info);

/* Bytes of device memory past the end of the last record that the kernels may read (the
 * LDS windows of pv_topn_names and the DNS pass load whole 16-B aligned windows of up to
 * 192 bytes from a record's start). Every d_recs buffer must be readable this far. */
#define PV_RECS_PAD 256

/* Process a block of records already resident in device memory. d_recs must be
 * readable for PV_RECS_PAD bytes past the last record. `stream` is a hipStream_t
 * (NULL = the context's own stream). Each manager (Net, DNS) shifts its own window on the
 * first of its own events at or after its next shift (AbstractMetricsManager::new_event,
 * src/AbstractMetricsManager.h:318-333); a batch that may hold a DNS shift is prescanned
 * for its DNS events first, and a batch with more than PV_MAX_SHIFTS (6) shifts of one
 * manager is processed as several device spans. Returns once the batch's status is read. */
int pv_process_device(pv_ctx *ctx, const uint8_t *d_recs, const uint32_t *d_offsets, const pv_index_info *info,
                      const uint32_t *sec_change_idx, const uint32_t *sec_change_sec, void *stream);

/* pv_index_records with the walk split over nthreads host threads (0 = default:
 * PV_HOST_THREADS, else the online CPUs up to 16); identical results. */
int pv_index_records_mt(const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets, uint64_t max_records,
                        uint32_t *sec_change_idx, uint32_t *sec_change_sec, uint32_t max_changes, pv_index_info *info,
                        uint32_t nthreads);

/* Process records in host memory, pipelined over 64 MiB chunks (PV_INGEST_CHUNK_MB). The
 * blob is copied to the device in fixed chunks (through pinned staging unless recs is
 * pinned, e.g. registered with pv_host_register) on two copy streams into a ring of device
 * buffers (PV_INGEST_RING, 3..8, default 4), ahead of the kernels; each chunk, joined to the previous batch's tail on
 * the device, is indexed there (pv_index_records_device's kernels) and processed as batches
 * that end at a ts_sec boundary. PV_INGEST_INDEX=host selects the host-walk pipeline
 * (parallel host index, H2D of records + offsets). Returns when every record has been
 * processed. */
int pv_process_host(pv_ctx *ctx, const uint8_t *recs, size_t bytes);
/* dnstap input: a Frame Streams file of dnstap.Dnstap protobuf frames (DnstapInputStream,
 * src/inputs/dnstap/DnstapInputStream.cpp:33-92) through both handlers' process_dnstap
 * (NetworkMetricsBucket::process_dnstap, net/v1/NetStreamHandler.cpp:549-620;
 * DnsMetricsBucket::process_dnstap, dns/v1/DnsStreamHandler.cpp:839-909; the managers at
 * :832-843 and :1376-1412). msg_type_mask is the DNS handler's "dnstap_msg_type" filter
 * (bit t: dnstap Message.Type t passes; 0 = no filter, :171-184,260-266): a message of
 * another type is a filtered DNS event. Timestamps: the response time of CLIENT / AUTH /
 * RESOLVER responses, the query time of their queries, else the wall clock. The v2 handlers'
 * dnstap paths (Net v2 process_dnstap, DNS v2 transactions per message-type direction) are built,
 * and the input's only_hosts filter is pv_set_dnstap_only_hosts. */
int pv_process_dnstap(pv_ctx *ctx, const uint8_t *frames, size_t bytes, uint32_t msg_type_mask);
/* The dnstap input proxy's "only_hosts" (DnstapInputEventProxy, src/inputs/dnstap/DnstapInputStream.h:
 * 96-146): comma-separated CIDRs, parsed with parse_host_specs' error texts; NULL clears. A message is
 * kept only when it has both addresses and one of them matches, with the reference's
 * match_subnet(..., std::string) reading the raw address bytes as text. */
int pv_set_dnstap_only_hosts(pv_ctx *ctx, const char *hosts);
/* Frame Streams decode only: data frames read and dnstap MESSAGE events in them. */
int pv_dnstap_count(const uint8_t *frames, size_t bytes, uint32_t *n_frames, uint32_t *n_events);

/* pcapng capture (PcapInputStream opens "pcap or pcapng", PcapInputStream.cpp:475-481, via
 * PcapPlusPlus / LightPcapNg) -> classic pcap records with nanosecond fractions (feed them
 * with pv_config.ts_nano = 1): Enhanced, Simple and obsolete Packet blocks of every section,
 * timestamps in each interface's if_tsresol units. All interfaces must share one linktype
 * (*linktype; PV_EUNSUPPORTED otherwise). out == NULL: sizes only; PV_ECAPACITY if out_cap is
 * too small; PV_EINVAL for a malformed file. Host function, no context. */
int pv_pcapng_records(const uint8_t *buf, size_t bytes, uint8_t *out, size_t out_cap, size_t *out_bytes,
                      uint32_t *linktype, uint64_t *n_records);

/* AF_PACKET TPACKET_V3 ingest: one ring block the kernel handed to user space (the block
 * walk of AFPacket::walk_block, src/inputs/pcap/afpacket.cpp:72-86) -> classic pcap records
 * with nanosecond fractions appended at out + *out_bytes (*out_bytes advanced, *n_records
 * incremented), for pv_process_host (pv_config.ts_nano = 1, linktype 1). Every packet takes
 * the block's ts_last_pkt, as the reference's RawPacket does (:81). The socket, ring mmap and
 * poll loop stay the caller's (CAP_NET_RAW). PV_EINVAL: a malformed block; PV_ECAPACITY: out
 * is full (nothing of this block's remaining packets is appended past out_cap). */
int pv_tpacket3_block_records(const uint8_t *block, size_t block_size, uint8_t *out, size_t out_cap, size_t *out_bytes,
                              uint64_t *n_records);

/* AF_PACKET live capture (visor::input::pcap::AFPacket, src/inputs/pcap/afpacket.cpp:22-262):
 * the TPACKET_V3 ring loop in front of pv_process_host. A capture thread waits on the ring
 * (poll), turns every block the kernel hands over into pcap records in a page-locked staging
 * buffer (pv_tpacket3_block_records) and gives the block back at once; a processing thread runs
 * pv_process_host on each full buffer (batch_bytes, or after flush_ms without a full one) while
 * the other fills. The context must be created with linktype 1 and ts_nano = 1. */
typedef struct pv_afpacket pv_afpacket;
typedef struct pv_afpacket_config {
    const char *interface;  /* "any" (default) or an interface name (AFPacket::set_interface) */
    int fanout_group_id;    /* -1: no fanout; else a PACKET_FANOUT_LB group (AFPacket::setup) */
    uint32_t block_size;    /* ring block bytes (0: 1 << 22, afpacket.h) */
    uint32_t frame_size;    /* 0: 1 << 11 */
    uint32_t num_blocks;    /* 0: 64 */
    const void *bpf_insns;  /* a compiled classic BPF program (struct sock_filter[]) or NULL: what
                               filter_try_compile hands to SO_ATTACH_FILTER (no libpcap here) */
    uint32_t bpf_len;       /* instructions */
    uint32_t batch_bytes;   /* staging bytes per pv_process_host call (0: 64 MiB) */
    uint32_t flush_ms;      /* a partial batch goes after this long without a new block (0: 100) */
} pv_afpacket_config;
typedef struct pv_afpacket_counters {
    uint64_t blocks, packets, batches, bytes;            /* ring blocks walked, packets, batches, record bytes */
    uint64_t kernel_packets, kernel_drops, kernel_freezes; /* PACKET_STATISTICS (tpacket_stats_v3), socket mode */
} pv_afpacket_counters;
/* Records of one staging buffer, in capture order; nonzero return stops the capture. */
typedef int (*pv_afpacket_sink)(void *user, const uint8_t *recs, size_t bytes, uint64_t n_records);
/* The socket, ring and fanout of AFPacket::AFPacket / set_socket_opts / setup. Needs CAP_NET_RAW
 * (PV_EUNSUPPORTED without it). Messages: pv_afpacket_last_error (this thread). */
int pv_afpacket_open(const pv_afpacket_config *cfg, pv_afpacket **out);
/* The same loop over a ring mapped by the caller: num_blocks blocks of block_size bytes laid out
 * as the kernel fills them (tpacket_block_desc + tpacket3_hdr packets); a block is the loop's
 * when its block_status has TP_STATUS_USER and is returned with TP_STATUS_KERNEL. wake_fd: an
 * eventfd the ring's producer signals (polled as the socket would be), or -1 to spin. */
int pv_afpacket_attach(uint8_t *ring, uint32_t block_size, uint32_t num_blocks, int wake_fd, const pv_afpacket_config *cfg,
                       pv_afpacket **out);
/* Capture on the calling thread until pv_afpacket_stop (from another thread), feeding sink;
 * returns the first sink / ring failure, 0 after a stop (the last partial batch delivered). */
int pv_afpacket_run(pv_afpacket *a, pv_afpacket_sink sink, void *user);
/* AFPacket::start_capture: the loop on its own thread feeding pv_process_host(ctx). */
int pv_afpacket_start(pv_afpacket *a, pv_ctx *ctx);
/* AFPacket::stop_capture: ends the loop (after delivering the partial batch); the loop's status. */
int pv_afpacket_stop(pv_afpacket *a);
int pv_afpacket_stats(pv_afpacket *a, pv_afpacket_counters *out);
void pv_afpacket_close(pv_afpacket *a);
const char *pv_afpacket_last_error(void);

/* Page-lock a host range so pv_process_host DMAs from it directly (hipHostRegister). */
int pv_host_register(void *ptr, size_t bytes);
int pv_host_unregister(void *ptr);
/* Accumulated ms of the host-memory path. Device index (default): [0] copy into pinned
 * staging (pageable source, producer thread), [1] waiting for a chunk's copy + its record
 * index on the device, [3] device processing, as seen by the calling thread. Host index
 * (PV_INGEST_INDEX=host): [0] copy + index (pageable), [1] index (pinned), [2] H2D enqueue,
 * [3] device processing. */
int pv_ingest_timing(pv_ctx *ctx, double *ms4, int reset);
/* Multi-GPU shard edges (one context per rank, contiguous shards in rank order).
 * pv_edge_export: this shard's DNS transaction stubs (queries open at its end, responses
 * that are the first event of their (flow, txid) in it, its DNS period shifts).
 * pv_edge_merge: given every rank's export (bufs[0..nranks)), pair this shard's stub
 * responses with the queries the earlier shards leave open and count the timeouts of
 * those queries at this shard's shifts, into this rank's buckets; call before the
 * bucket all-reduce. Replaces the single-stream TransactionManager continuity
 * (libs/visor_transaction/TransactionManager.h:51-106) across shard boundaries. */
int pv_edge_export(pv_ctx *ctx, uint8_t **buf, size_t *bytes);
int pv_edge_merge(pv_ctx *ctx, const uint8_t *const *bufs, const size_t *sizes, uint32_t nranks, uint32_t my_rank);
/* Sharded top_slow. A slow transaction is counted against the p90 of the bucket that closed
 * at the last DNS shift (DnsMetricsManager::on_period_shift, dns/v1/DnsStreamHandler.h:252-267),
 * a bucket that spans several shards. With pv_set_slow_defer(ctx, 1) (before the first batch;
 * DNS v1) a rank keeps every slow candidate (valid, deep transaction of known direction,
 * edge pairs included) with its response record instead of checking it against its own
 * shard's p90. At the merge, after pv_edge_merge and before pv_values_merge / the top-N
 * exchange: pv_slow_values_export (this rank's transaction times per DNS period ordinal),
 * all-gather, pv_slow_finish (each live-window period's thresholds from every rank's values,
 * then this rank's candidates of those periods into their top_slow tables). */
int pv_set_slow_defer(pv_ctx *ctx, int defer);
/* Shard-edge transactions of such a run, carried in rank order (replaces pv_edge_export /
 * pv_edge_merge there): `in` = the DNS queries the earlier shards leave open (the previous
 * rank's *out; empty for rank 0). Each meets the first event of its (flow, txid) in this shard
 * as the TransactionManager would (libs/visor_transaction/TransactionManager.h:51-106): a
 * response pairs with it (counted, its times and top_slow candidate kept), a query overwrites
 * it, a DNS shift of this shard at or after ttl + its start purges it first (a time-out there,
 * dns/v1/DnsStreamHandler.h:252-267). *out: the queries still open at this shard's end, the
 * earlier shards' survivors and this shard's own (pv_free). */
int pv_edge_carry(pv_ctx *ctx, const uint8_t *in, size_t in_bytes, uint8_t **out, size_t *out_bytes);
/* The end of the capture: the next pv_process_host / pv_process_device call holds the capture's
 * last records, and after them every TCP connection still open is closed, as
 * TcpReassembly::closeAllConnections does when a pcap file ends and when the input stops
 * (src/inputs/pcap/PcapInputStream.cpp:522, :244): a connection's held out-of-order fragments are
 * delivered behind their missing-data markers and the DNS messages that completes are counted at
 * the connection's end time, with the direction the input cached for its last packet
 * (_packet_dir_cache, :399-416). on = 0 disarms it. The flag applies to that call's final batch
 * (pv_process_host cuts its data into batches) and is cleared by the call. */
int pv_set_end_of_capture(pv_ctx *ctx, int on);
/* Sharded runs, before the merge: what this shard holds that a merge step exchanges.
 * open_queries: the DNS queries it leaves open at its end, before any edge carry (an upper bound:
 * the carried list, one entry per event); a merge in which every rank reports 0 has no transaction
 * across a shard edge, so the edge exchange is skipped, else it starts at the first rank that
 * reports one (TransactionManager.h:51-106: a query is the only event a later shard can complete).
 * xact_values: its DNS transaction values (quantile and top_slow inputs); with 0 on every rank the
 * distributed selections (pv_comm_slow_finish, pv_comm_values_select) have nothing to select. */
int pv_merge_hints(pv_ctx *ctx, uint64_t *open_queries, uint64_t *xact_values);
int pv_slow_values_export(pv_ctx *ctx, uint8_t **buf, size_t *bytes);
int pv_slow_finish(pv_ctx *ctx, const uint8_t *const *bufs, const size_t *sizes, uint32_t nranks);
/* Quantile inputs of the live window, (slot, kind, value) records, for the merge of the
 * dns_xact_* quantiles across ranks (DnsMetricsBucket::specialized_merge of the KLL
 * sketches, src/handlers/dns/v1/DnsStreamHandler.cpp:692). */
int pv_values_export(pv_ctx *ctx, uint8_t **buf, size_t *bytes);
int pv_values_merge(pv_ctx *ctx, const uint8_t *buf, size_t bytes);
/* Live slots of one manager (part 0 = Net "packets", 1 = DNS) with their bucket start
 * seconds, newest first. */
int pv_window_periods(pv_ctx *ctx, int part, uint32_t *slots, int64_t *start_sec, uint32_t max_n, uint32_t *n);
/* Sharded runs (one context per rank, contiguous shards): shifts of one manager whose shifting
 * event lies in another rank's shard, applied in order as window operations only (an empty
 * bucket opens at each threshold second). Call with the earlier ranks' shifts before the first
 * batch and with the later ranks' shifts after the last, so every rank's window holds the same
 * periods in the same slots (the global period table). */
int pv_advance_windows(pv_ctx *ctx, int part, const int64_t *thresh, uint32_t n);
/* The seconds (stream order, each once) in which a device batch holds a DNS event (a UDP
 * datagram on a DNS port that the input predicates pass): what the ranks exchange to compute
 * the DNS manager's global shifts. Does not touch the buckets. */
int pv_dns_event_seconds(pv_ctx *ctx, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                         const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n);
/* The same over records in host memory (staged through the ingest chunks). */
/* Deep sampling across shards: the DNS manager's draws (unfiltered DNS events, TCP messages
 * included) the last pv_dns_event_seconds_host call counted (0 at deep_sample_rate 100), and
 * the generators of a rank stepped past the earlier shards' draws before its first batch:
 * net_draws = their records, dns_draws = the sum of their pv_plan_dns_draws
 * (AbstractMetricsManager::new_event's per-manager jsf32 draws, src/AbstractMetricsManager.h:318-323). */
int pv_plan_dns_draws(pv_ctx *ctx, uint64_t *draws);
int pv_sample_skip(pv_ctx *ctx, uint64_t net_draws, uint64_t dns_draws);
int pv_dns_event_seconds_host(pv_ctx *ctx, const uint8_t *recs, size_t bytes, int64_t *secs, uint32_t max, uint32_t *n);
/* Record cuts of a capture into `world` contiguous shards (cuts[0..world], cuts[world] = n):
 * about equal sizes, each cut at a record boundary that no DNS-over-TCP flow (a TCP packet with
 * a DNS port, keyed as the TCP stage keys it) spans, so DNS over TCP across shard edges matches a
 * single pass (PcapInputStream.cpp:254-283, 429-465 reassemble per connection in capture order).
 * offs: the records' byte offsets in recs (pv_index_records). */
int pv_shard_cuts(const uint8_t *recs, size_t bytes, const uint32_t *offs, uint64_t n, uint32_t linktype, uint32_t ts_nano,
                  uint32_t world, uint64_t *cuts);


int pv_set_start_tstamp(pv_ctx *ctx, int64_t sec, int64_t nsec);
int pv_set_end_tstamp(pv_ctx *ctx, int64_t sec, int64_t nsec);
int pv_synchronize(pv_ctx *ctx);
/* Clear every bucket and all transaction state (a fresh handler). */
int pv_reset(pv_ctx *ctx);

/* JSON for schema keys "packets" and "dns": {"packets":{...},"dns":{...}}.
 * merged == 0: bucket `period` (0 = live); merged != 0: merge the `period` most
 * recent buckets (window_merged_json). *out is malloc'd; free with pv_free. */
int pv_window_json(pv_ctx *ctx, uint32_t period, int merged, char **out);
void pv_free(void *p);

/* Prometheus text exposition of bucket `period` (0 = live) of the v1 handlers selected by
 * `handlers` (PV_HANDLER_NET: "packets_*", PV_HANDLER_DNS: "dns_*"; both: Net then DNS), in
 * the reference's metric order, names, HELP texts and number formatting; labels: the static
 * labels, then these n_labels added ones (each set in key order). Rates are timer-driven and
 * not kept: nothing is written for them, as for an empty Rate. The v2 handlers are refused
 * (PV_EUNSUPPORTED). *out: pv_free. */
#define PV_HANDLER_NET 1u
#define PV_HANDLER_DNS 2u
/* period argument of pv_window_prometheus / pv_window_opentelemetry: what
 * StreamMetricsHandler::window_prometheus / window_opentelemetry read (src/StreamHandler.h:226-247):
 * bucket 1 of a handler whose manager holds more than one bucket, else bucket 0 */
#define PV_PERIOD_AUTO 0xFFFFFFFFu
int pv_window_prometheus(pv_ctx *ctx, uint32_t period, uint32_t handlers, const char *const *label_keys,
                         const char *const *label_values, uint32_t n_labels, char **out);
/* OpenTelemetry metrics of bucket `period` of the selected v1 handlers, as the protobuf
 * wire bytes of the ScopeMetrics fields the reference's primitives fill (the repeated
 * `metrics`, in the handlers' order): append them to a ScopeMetrics with MergeFromString.
 * Attributes: the n_labels added labels. *out: pv_free. */
int pv_window_opentelemetry(pv_ctx *ctx, uint32_t period, uint32_t handlers, const char *const *label_keys,
                            const char *const *label_values, uint32_t n_labels, uint8_t **out, size_t *bytes);
/* Process-wide label on every Prometheus sample (Metric::add_static_label). */
int pv_add_static_label(const char *key, const char *value);

/* Heartbeat (PcapInputEventProxy::heartbeat_signal -> StreamMetricsHandler::check_period_shift,
 * src/StreamHandler.h:254-257, src/AbstractMetricsManager.h:462-470; wired in
 * net/v1/NetStreamHandler.cpp:99-102 and dns/v1/DnsStreamHandler.cpp:219-222): each manager
 * whose next shift second the stamp has reached shifts its window with no event (num_periods
 * > 1); the DNS manager's on_period_shift (dns/v1/DnsStreamHandler.h:252-267) times out the
 * open transactions the stamp expires into the new live bucket and takes the top_slow p90
 * thresholds from the bucket just closed. A context that has seen no record ignores it. */
int pv_check_period_shift(pv_ctx *ctx, int64_t sec, int64_t nsec);

/* External metrics buckets: the bucket half of the handler object
 * (StreamHandler::merge / window_json(j, bucket) / window_prometheus(out, bucket, labels) /
 * window_opentelemetry(scope, bucket, labels), src/StreamHandler.h:72-77,221-269), which a policy
 * uses to fold like handlers across taps (Policy::_get_merged_buckets, src/Policies.cpp:420-446).
 * A pv_bucket is a host-side snapshot of one handler's bucket (handler = PV_HANDLER_NET: the
 * Net v1 part and, when attached, Net v2's; PV_HANDLER_DNS: DNS v1 or v2, as configured). */
typedef struct pv_bucket pv_bucket;
/* StreamMetricsHandler::merge(bucket, period, prometheus, merged): *bucket == NULL -> a new bucket
 * holding this context's bucket `period` (merged: the fold of its `period` newest buckets,
 * multiple_merge), as simple_merge / multiple_merge create it (src/AbstractMetricsManager.h:649-706);
 * *bucket != NULL (a bucket of the same handler, from any context) -> this context's bucket folded
 * into it with Aggregate::SUM (quantiles summed p-wise, src/Metrics.h:356-372). prometheus != 0:
 * period 1 when the manager holds more than one bucket, else 0, never merged. Period errors
 * carry the reference's PeriodException texts. */
int pv_bucket_merge(pv_ctx *ctx, uint32_t handler, pv_bucket **bucket, uint32_t period, int prometheus, int merged);
/* window_external_json / _prometheus / _opentelemetry (src/AbstractMetricsManager.h:565-599),
 * rendered with ctx's handler config (groups, topn_count, percentile threshold). JSON:
 * {"packets": {...}} or {"dns": {...}}. *out: pv_free. */
int pv_bucket_json(pv_ctx *ctx, const pv_bucket *bucket, char **out);
int pv_bucket_prometheus(pv_ctx *ctx, const pv_bucket *bucket, const char *const *label_keys,
                         const char *const *label_values, uint32_t n_labels, char **out);
int pv_bucket_opentelemetry(pv_ctx *ctx, const pv_bucket *bucket, const char *const *label_keys,
                            const char *const *label_values, uint32_t n_labels, uint8_t **out, size_t *bytes);
void pv_bucket_free(pv_bucket *bucket);

/* Device-state regions of the live window, for a multi-GPU reduce:
 *   SUM region: uint64 counters and dense tables (all-reduce SUM)
 *   MIN region: int64 CPC first-occurrence global record indices (all-reduce MIN)
 * Global record index = pv_set_global_base() + records processed before; ranks
 * that process contiguous shards set their shard's first global record index. */
int pv_state_regions(pv_ctx *ctx, void **sum_ptr, size_t *sum_bytes, void **min_ptr, size_t *min_bytes);
int pv_set_global_base(pv_ctx *ctx, uint64_t base);
/* The device regions of both live windows a multi-GPU reduce combines, in a fixed order
 * (identical on every rank whose windows hold the same periods): per Net slot its net part,
 * per DNS slot its dns part, of the SUM words (uint64, all-reduce SUM) and of the MIN words
 * (int64 CPC first-occurrence indices, all-reduce MIN). */
enum pv_reduce_op { PV_REDUCE_SUM = 0, PV_REDUCE_MIN = 1 };
typedef struct pv_region {
    void *ptr;      /* device pointer */
    uint64_t words; /* 64-bit words */
    uint32_t op;    /* pv_reduce_op */
    uint32_t pad;
} pv_region;
int pv_window_regions(pv_ctx *ctx, pv_region *regions, uint32_t max, uint32_t *n);

/* ---- RCCL over xGMI: one communicator per context (one process or thread per GPU).
 * Replaces the reference's single-process merge of per-input handler buckets
 * (AbstractMetricsManager::window_merged_json, src/AbstractMetricsManager.h:601-647, and
 * the Policies' handler merge, src/Policies.cpp:420-446) for a context sharded across GPUs:
 * SUM / MIN all-reduce of the live window regions in device memory, and an all-gather of
 * host byte blobs (top-N lists, shard-edge stubs, quantile inputs). */
#define PV_COMM_ID_BYTES 128
/* ncclGetUniqueId: called on one rank, the bytes passed to every rank out of band */
int pv_comm_unique_id(uint8_t id[PV_COMM_ID_BYTES]);
/* ncclCommInitRank on the context's device */
int pv_comm_init(pv_ctx *ctx, const uint8_t id[PV_COMM_ID_BYTES], int nranks, int rank);
/* in-place all-reduce of every region pv_window_regions lists (u64 SUM / i64 MIN), one
 * RCCL group on the context's stream; returns after the reduction completed */
int pv_comm_allreduce_window(pv_ctx *ctx);
/* all-gather of one host byte blob per rank: *out (pv_free) holds the blobs of ranks
 * 0..n-1 back to back, sizes[r] their lengths (sizes has nranks entries) */
int pv_comm_allgather(pv_ctx *ctx, const void *buf, size_t bytes, uint8_t **out, uint64_t *sizes);
int pv_comm_destroy(pv_ctx *ctx);
/* Compact the top-N tables of all live buckets into a host buffer of
 * (slot, metric, key, count, name) records (see pvgpu_topn_rec) for exchange;
 * pv_merge_topn adds such records from another rank into this context's view. */
int pv_export_topn(pv_ctx *ctx, uint8_t **buf, size_t *bytes);
int pv_merge_topn(pv_ctx *ctx, const uint8_t *buf, size_t bytes);

/* ---- Multi-GPU top-N merge on the device (the frequent-items merge of
 * AbstractMetricsBucket::merge, src/AbstractMetricsManager.h:177-195 / src/Metrics.h:534-538,
 * over shards of one stream). Every table's regions are split over the ranks in contiguous
 * blocks; each rank ships the live entries (key, count) of the regions others own to their
 * owners, which merge them into their regions on the device (pv_topn_merge). Names are not
 * shipped: the read path collects every owner's leading entries per metric and fetches the
 * names of those from whichever rank holds them. Collective: every rank calls each step with
 * windows holding the same periods (the global period plan).
 *   pv_comm_merge_topn: the whole exchange over the context's RCCL communicator (device to
 *     device, one count round and one point-to-point round);
 *   pv_topn_x_export / pv_topn_x_import: the same through host blobs (any transport): export
 *     gives this rank's blob (pv_free), import takes every rank's blob in rank order.
 * Afterwards the context's top-N view is its own regions until pv_topn_x_view installs the
 * merged lists:
 *   pv_topn_x_candidates: this rank's leading entries per metric (topn_count, and every entry
 *     tied with the last), with the names it holds (blob, pv_free);
 *   pv_topn_x_names: given every rank's candidate blob, the names this rank holds for the
 *     candidates that came without one (blob, pv_free);
 *   pv_topn_x_view: every rank's candidate and name blobs: the merged top-N lists. */
int pv_comm_merge_topn(pv_ctx *ctx);
int pv_topn_x_export(pv_ctx *ctx, uint32_t ranks, uint32_t rank, uint8_t **blob, size_t *bytes);
int pv_topn_x_import(pv_ctx *ctx, uint32_t ranks, uint32_t rank, const uint8_t *const *blobs, const size_t *sizes);
int pv_topn_x_candidates(pv_ctx *ctx, uint8_t **blob, size_t *bytes);
int pv_topn_x_names(pv_ctx *ctx, const uint8_t *const *cands, const size_t *sizes, uint32_t n, uint8_t **blob, size_t *bytes);
int pv_topn_x_view(pv_ctx *ctx, const uint8_t *const *cands, const size_t *csizes, const uint8_t *const *names,
                   const size_t *nsizes, uint32_t n);

/* Quantile inputs across shards without shipping the values (replaces pv_values_export /
 * pv_values_merge for merged reads): an exact radix selection, eight passes of 256-bin group
 * histograms summed over the ranks, gives per live DNS slot and value kind the count, p50, p90,
 * p95, p99 and maximum of the union of the shards' transaction values (the KLL inclusive rank rule
 * of Quantile, src/Metrics.h:334-481), and for the time kinds the counts at the histogram points
 * (Histogram, :189-327); the merged view reads them instead of this rank's values. Collective.
 * pv_values_x_select sums through the caller's all-reduce (op 0 SUM, 1 MAX; return 0 on success),
 * pv_comm_values_select through the context's RCCL communicator. */
typedef int (*pv_allreduce_fn)(uint64_t *buf, size_t n, int op, void *user);
int pv_values_x_select(pv_ctx *ctx, pv_allreduce_fn allreduce, void *user);
int pv_comm_values_select(pv_ctx *ctx);
/* pv_slow_finish without shipping the transaction times: each DNS period's p90 (the bucket
 * that closed at each shift, DnsMetricsManager::on_period_shift, dns/v1/DnsStreamHandler.h:
 * 252-267) by the same distributed selection, then this rank's deferred candidates judged.
 * Collective (every rank, pv_set_slow_defer contexts). */
int pv_slow_x_finish(pv_ctx *ctx, pv_allreduce_fn allreduce, void *user);
int pv_comm_slow_finish(pv_ctx *ctx);

/* Device time of the Net-pass kernel (pv_net_kernel): the start and end stamps of its dispatch
 * packet (HIP events of hipExtLaunchKernelGGL), summed over the stamped launches since the last
 * reset: total milliseconds and number of stamped launches. Which launches are stamped is
 * pv_set_kernel_timing's: every `every`-th batch, 0 (the default) none. A stamped dispatch
 * leaves the device idle for ~14 us around it, so a measurement samples. */
int pv_set_kernel_timing(pv_ctx *ctx, uint32_t every);
/* The Net-pass kernel the last span launched ("pv_net_kernel_reg", "pv_net_kernel", ...): the
 * name rocprofv3 reports for the launches pv_kernel_timing times. */
const char *pv_net_kernel_name(pv_ctx *ctx);
int pv_kernel_timing(pv_ctx *ctx, double *total_ms, uint64_t *launches, int reset);

#ifdef __cplusplus
}
#endif
#endif /* PVGPU_H */
