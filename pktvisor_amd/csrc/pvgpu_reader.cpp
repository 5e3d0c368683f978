// SPDX-License-Identifier: MPL-2.0
// pvgpu-reader — GPU counterpart of cmd/pktvisor-reader/main.cpp:86-258 for the
// net + dns handlers: pvgpu-reader [-H HOST_SPEC] [--periods N] FILE
// Prints {"<N>m": {"packets": {...}, "dns": {...}}} like the reference.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "../../include/pvgpu.h"

int main(int argc, char **argv)
{
    std::string host, file;
    unsigned periods = 5;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "-H" && i + 1 < argc) host = argv[++i];
        else if (a == "--periods" && i + 1 < argc) periods = (unsigned)atoi(argv[++i]);
        else file = a;
    }
    std::ifstream f(file, std::ios::binary);
    if (!f) { fprintf(stderr, "Cannot open pcap/pcapng file\n"); return 1; }
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (buf.size() < 24) { fprintf(stderr, "Cannot open pcap/pcapng file\n"); return 1; }
    uint32_t magic, linktype;
    memcpy(&magic, buf.data(), 4);
    memcpy(&linktype, buf.data() + 20, 4);
    if (magic != 0xa1b2c3d4 && magic != 0xa1b23c4d) { fprintf(stderr, "unsupported pcap format\n"); return 1; }
    pv_config cfg{};
    cfg.host_spec = host.empty() ? nullptr : host.c_str();
    cfg.num_periods = periods;
    cfg.linktype = linktype;
    cfg.ts_nano = magic == 0xa1b23c4d;
    cfg.device = -1;
    uint64_t nrec = 0;
    for (size_t p = 24; p + 16 <= buf.size(); nrec++) { uint32_t l; memcpy(&l, &buf[p + 8], 4); p += 16 + l; }
    cfg.max_records = nrec ? nrec : 1;
    pv_ctx *ctx = nullptr;
    int rc = pv_create(&cfg, &ctx);
    if (rc) { fprintf(stderr, "Fatal error: %s\n", ctx ? pv_last_error(ctx) : "pv_create"); pv_destroy(ctx); return 1; }
    rc = pv_process_host(ctx, buf.data() + 24, buf.size() - 24);
    if (!rc && nrec) {
        // end_tstamp_signal with the last record (PcapInputStream.cpp:514-517)
        size_t p = 24, last = 24;
        while (p + 16 <= buf.size()) { uint32_t l; memcpy(&l, &buf[p + 8], 4); last = p; p += 16 + l; }
        uint32_t s, fr;
        memcpy(&s, &buf[last], 4);
        memcpy(&fr, &buf[last + 4], 4);
        pv_set_end_tstamp(ctx, s, cfg.ts_nano ? fr : (int64_t)fr * 1000);
    }
    char *out = nullptr;
    if (!rc) rc = pv_window_json(ctx, periods == 1 ? 0 : periods, periods == 1 ? 0 : 1, &out);
    if (rc) { fprintf(stderr, "Fatal error: %s\n", pv_last_error(ctx)); pv_destroy(ctx); return 1; }
    printf("{\"%um\":%s}\n", periods == 1 ? 1 : periods, out);
    pv_free(out);
    pv_destroy(ctx);
    return 0;
}
