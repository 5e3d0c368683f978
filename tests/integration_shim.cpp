// The pv_* calls of INTEGRATION.md's plugin shim and bindings, with the argument types the shim
// passes, compiled against include/pvgpu.h on the CPU (tests/test_integration_doc.py): a
// maintainer binding from the header and the document gets calls that type-check. Never run.
#include "../include/pvgpu.h"

#include <cstdint>
#include <cstdlib>
#include <vector>

namespace {
struct Staging {
    pv_ctx *ctx = nullptr;
    std::vector<uint8_t> staging;
};
int sink(void *, const uint8_t *, size_t, uint64_t) { return 0; }
int ar(uint64_t *, size_t, int, void *) { return 0; }
}

int integration_shim_calls(Staging &g, const char *qtype, uint64_t cache_limit, int64_t sec, int64_t nsec)
{
    int rc = 0;
    pv_config c{};
    pv_ctx *ctx = nullptr;
    rc |= pv_create(&c, &ctx);
    g.ctx = ctx;
    // section 1: the handler shim
    rc |= pv_set_tcp_reassembly_limit(ctx, cache_limit);
    rc |= pv_set_tcp_exact_lru(ctx, 1);
    pv_dns_filters f{};
    f.answer_count = -1;
    uint32_t v = 0;
    rc |= pv_dns_code(1, qtype, &v);
    f.qtypes[f.n_qtypes++] = (uint16_t)v;
    rc |= pv_set_dns_filters(ctx, &f);
    rc |= pv_process_host(ctx, g.staging.data(), g.staging.size());
    rc |= pv_set_start_tstamp(ctx, sec, nsec);
    rc |= pv_set_end_tstamp(ctx, sec, nsec);
    rc |= pv_check_period_shift(ctx, sec, nsec);
    char *out = nullptr;
    rc |= pv_window_json(ctx, 5u, 1, &out);
    pv_free(out);
    std::vector<const char *> k{"instance"}, val{"a"};
    char *text = nullptr;
    rc |= pv_window_prometheus(ctx, PV_PERIOD_AUTO, PV_HANDLER_NET, k.data(), val.data(), (uint32_t)k.size(), &text);
    pv_free(text);
    uint8_t *pb = nullptr;
    size_t n = 0;
    rc |= pv_window_opentelemetry(ctx, PV_PERIOD_AUTO, PV_HANDLER_DNS, k.data(), val.data(), (uint32_t)k.size(), &pb, &n);
    pv_free(pb);
    pv_bucket *b = nullptr;
    rc |= pv_bucket_merge(ctx, PV_HANDLER_NET, &b, 0u, 0, 1);
    rc |= pv_bucket_json(ctx, b, &out);
    rc |= pv_bucket_prometheus(ctx, b, k.data(), val.data(), (uint32_t)k.size(), &text);
    rc |= pv_bucket_opentelemetry(ctx, b, k.data(), val.data(), (uint32_t)k.size(), &pb, &n);
    pv_bucket_free(b);
    rc |= pv_add_static_label("instance", "a");
    const char *err = pv_last_error(ctx);
    (void)err;
    // dnstap, BPF, AF_PACKET
    rc |= pv_process_dnstap(ctx, g.staging.data(), g.staging.size(), 1u << 5 | 1u << 6);
    pv_bpf_insn prog[1] = {{0x06, 0, 0, 0xffff}};
    rc |= pv_set_bpf(ctx, prog, 1);
    pv_afpacket_config ac{};
    ac.bpf_insns = prog;
    ac.bpf_len = 1;
    pv_afpacket *ring = nullptr;
    rc |= pv_afpacket_open(&ac, &ring);
    rc |= pv_afpacket_start(ring, ctx);
    rc |= pv_afpacket_run(ring, sink, nullptr);
    pv_afpacket_counters cnt{};
    rc |= pv_afpacket_stats(ring, &cnt);
    rc |= pv_afpacket_stop(ring);
    pv_afpacket_close(ring);
    std::vector<uint8_t> map(1 << 16);
    rc |= pv_afpacket_attach(map.data(), 1u << 16, 1u, -1, &ac, &ring);
    // multi-GPU (section "Multi-GPU")
    uint8_t id[PV_COMM_ID_BYTES];
    rc |= pv_comm_unique_id(id);
    rc |= pv_comm_init(ctx, id, 8, 0);
    rc |= pv_set_slow_defer(ctx, 1);
    rc |= pv_comm_slow_finish(ctx);
    rc |= pv_slow_x_finish(ctx, ar, nullptr);
    rc |= pv_comm_allreduce_window(ctx);
    rc |= pv_comm_merge_topn(ctx);
    uint8_t *blob = nullptr;
    size_t bytes = 0;
    rc |= pv_topn_x_export(ctx, 8u, 0u, &blob, &bytes);
    const uint8_t *blobs[1] = {blob};
    const size_t sizes[1] = {bytes};
    rc |= pv_topn_x_import(ctx, 1u, 0u, blobs, sizes);
    rc |= pv_topn_x_candidates(ctx, &blob, &bytes);
    rc |= pv_topn_x_names(ctx, blobs, sizes, 1u, &blob, &bytes);
    rc |= pv_topn_x_view(ctx, blobs, sizes, blobs, sizes, 1u);
    rc |= pv_comm_values_select(ctx);
    rc |= pv_values_x_select(ctx, ar, nullptr);
    pv_region regions[64];
    uint32_t nr = 0;
    rc |= pv_window_regions(ctx, regions, 64u, &nr);
    rc |= pv_comm_destroy(ctx);
    pv_destroy(ctx);
    return rc;
}
