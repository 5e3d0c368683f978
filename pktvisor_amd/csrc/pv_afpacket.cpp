// SPDX-License-Identifier: MPL-2.0
// pv_afpacket.cpp — the AF_PACKET TPACKET_V3 live-capture input in front of pv_process_host.
//
// Reference: visor::input::pcap::AFPacket (src/inputs/pcap/afpacket.cpp:22-262, afpacket.h):
// a raw socket with PACKET_VERSION = TPACKET_V3, promiscuous membership, an optional classic BPF
// program (SO_ATTACH_FILTER + SO_LOCK_FILTER), PACKET_RX_RING (tpacket_req3: 60 ms block retire
// timeout, RX hash), the ring mmap'ed, bound to the interface, optional PACKET_FANOUT_LB group; a
// capture thread polls the socket, walks each block the kernel hands to user space
// (TP_STATUS_USER), hands every packet on with the block's ts_last_pkt (walk_block) and gives
// the block back (flush_block: TP_STATUS_KERNEL).
//
// MI355X shape: the capture thread does no per-packet work beyond the copy. Each block is
// turned into classic pcap records (pv_tpacket3_block_records) appended to a page-locked
// staging buffer and retired at once; a full buffer (batch_bytes, or flush_ms without a full
// one) goes to a processing thread that calls pv_process_host (H2D + the device record index +
// the kernels) while the capture thread fills the other buffer. The kernel ring absorbs
// bursts while both buffers are busy (its drops are the PACKET_STATISTICS counters).
//
// pv_afpacket_attach runs the same loop over a ring the caller maps (another process's ring, or
// a memory-backed one in tests), with an fd the ring's producer makes readable to wake it.
// Filter-expression compilation (libpcap's pcap_compile in filter_try_compile) is not in this
// image: a filter comes in already compiled, as struct sock_filter[].
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <arpa/inet.h>
#include <linux/filter.h>
#include <linux/if_packet.h>
#include <net/ethernet.h>
#include <net/if.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include "../../include/pvgpu.h"

namespace {
thread_local char g_err[256];
int fail(int rc, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return rc;
}
int sink_process_host(void *user, const uint8_t *recs, size_t bytes, uint64_t)
{
    return pv_process_host(static_cast<pv_ctx *>(user), recs, bytes);
}
} // namespace

struct pv_afpacket {
    int fd = -1;      // the packet socket (pv_afpacket_open) or -1
    int wake_fd = -1; // attach mode: readable when the ring's producer released a block
    uint8_t *map = nullptr;
    size_t map_bytes = 0;
    bool own_map = false;
    uint32_t block_size = 0, num_blocks = 0;
    size_t batch_bytes = 0;
    uint32_t flush_ms = 0;
    std::atomic<bool> running{false};
    std::thread cap_thread;
    // staging: two page-locked buffers, one filling, one with the processing thread
    std::vector<uint8_t> stage[2];
    bool registered[2] = {false, false};
    size_t used[2] = {0, 0};
    uint64_t nrec[2] = {0, 0};
    int filling = 0;
    // processing thread
    std::thread worker;
    std::mutex m;
    std::condition_variable cv;
    int pending = -1; // staging buffer handed over, -1 none
    bool busy = false, quit = false;
    int rc = 0; // first failure of the loop or the sink
    pv_afpacket_sink sink = nullptr;
    void *user = nullptr;
    // counters
    std::atomic<uint64_t> blocks{0}, packets{0}, batches{0}, bytes{0};
    std::atomic<uint64_t> drops{0}, kpackets{0}, freezes{0}; // read_stats runs on the capture and caller threads

    ~pv_afpacket()
    {
        for (int b = 0; b < 2; b++)
            if (registered[b]) pv_host_unregister(stage[b].data());
        if (own_map && map) munmap(map, map_bytes);
        if (fd >= 0) close(fd);
    }
    void set_rc(int r)
    {
        std::lock_guard<std::mutex> g(m);
        if (!rc) rc = r;
    }
    void work()
    {
        for (;;) {
            int b;
            bool failed;
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return pending >= 0 || quit; });
                if (pending < 0) return;
                b = pending;
                pending = -1;
                busy = true;
                failed = rc != 0;
            }
            // after a failure the capture is ending: buffers still handed over are dropped
            const int r = failed ? 0 : sink(user, stage[b].data(), used[b], nrec[b]);
            if (!failed) {
                batches++;
                bytes += used[b];
            }
            {
                std::lock_guard<std::mutex> g(m);
                if (r && !rc) rc = r;
                used[b] = 0;
                nrec[b] = 0;
                busy = false;
            }
            cv.notify_all();
        }
    }
    // hand the filling buffer to the processing thread (waiting for it to take the last one)
    void flush()
    {
        if (!used[filling]) return;
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return pending < 0 && !busy; });
        pending = filling;
        filling ^= 1;
        g.unlock();
        cv.notify_all();
    }
    void drain()
    {
        flush();
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return pending < 0 && !busy; });
    }
    std::mutex stats_m; // PACKET_STATISTICS resets on read: one reader at a time
    void read_stats()
    {
        std::lock_guard<std::mutex> g(stats_m);
        if (fd < 0) return;
        tpacket_stats_v3 st{};
        socklen_t len = sizeof st;
        if (getsockopt(fd, SOL_PACKET, PACKET_STATISTICS, &st, &len) == 0) { // counters reset on read
            kpackets += st.tp_packets;
            drops += st.tp_drops;
            freezes += st.tp_freeze_q_cnt;
        }
    }
    // AFPacket::start_capture's loop (afpacket.cpp:214-243), batching into the staging buffers
    void capture()
    {
        uint32_t cur = 0;
        auto last = std::chrono::steady_clock::now();
        pollfd pfd{};
        pfd.fd = fd >= 0 ? fd : wake_fd;
        pfd.events = POLLIN | POLLERR;
        const int tmo = flush_ms ? (int)flush_ms : 100;
        while (running.load(std::memory_order_relaxed)) {
            {
                std::lock_guard<std::mutex> g(m);
                if (rc) break;
            }
            auto *bd = reinterpret_cast<tpacket_block_desc *>(map + (size_t)cur * block_size);
            const uint32_t status = __atomic_load_n(&bd->hdr.bh1.block_status, __ATOMIC_ACQUIRE);
            if (!(status & TP_STATUS_USER)) {
                const auto now = std::chrono::steady_clock::now();
                if (used[filling] && std::chrono::duration_cast<std::chrono::milliseconds>(now - last).count() >= tmo) {
                    flush();
                    last = now;
                }
                if (pfd.fd >= 0) {
                    pfd.revents = 0;
                    poll(&pfd, 1, tmo);
                    if (fd < 0 && (pfd.revents & POLLIN)) {
                        uint64_t v; // an eventfd: one read takes its whole count
                        if (read(wake_fd, &v, sizeof v) < 0) {
                        }
                    }
                } else {
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
                }
                continue;
            }
            // walk_block: the block's packets as pcap records; a block that does not fit the
            // filling buffer starts the next one (a block's records are smaller than the block)
            size_t o = used[filling];
            uint64_t nb = 0;
            int r = pv_tpacket3_block_records(map + (size_t)cur * block_size, block_size, stage[filling].data(),
                                              stage[filling].size(), &o, &nb);
            if (r == PV_ECAPACITY) {
                flush();
                last = std::chrono::steady_clock::now();
                o = used[filling];
                nb = 0;
                r = pv_tpacket3_block_records(map + (size_t)cur * block_size, block_size, stage[filling].data(),
                                              stage[filling].size(), &o, &nb);
            }
            if (r) {
                set_rc(fail(r, "malformed TPACKET_V3 block %u", cur));
                break;
            }
            used[filling] = o;
            nrec[filling] += nb;
            packets += nb;
            blocks++;
            __atomic_store_n(&bd->hdr.bh1.block_status, (uint32_t)TP_STATUS_KERNEL, __ATOMIC_RELEASE); // flush_block
            cur = (cur + 1) % num_blocks;
            if (used[filling] >= batch_bytes) {
                flush();
                last = std::chrono::steady_clock::now();
            }
        }
        drain();
        read_stats();
    }
    int init_staging()
    {
        const size_t cap = std::max<size_t>(batch_bytes, block_size) + block_size;
        for (int b = 0; b < 2; b++) {
            stage[b].assign(cap, 0);
            // page-locked so pv_process_host DMAs straight from it; best effort (a CPU sink needs none)
            registered[b] = pv_host_register(stage[b].data(), cap) == 0;
        }
        return 0;
    }
};

extern "C" {

const char *pv_afpacket_last_error(void) { return g_err; }

static void apply_defaults(const pv_afpacket_config *cfg, pv_afpacket *a)
{
    a->block_size = cfg && cfg->block_size ? cfg->block_size : 1u << 22; // afpacket.h defaults
    a->num_blocks = cfg && cfg->num_blocks ? cfg->num_blocks : 64;
    a->batch_bytes = cfg && cfg->batch_bytes ? cfg->batch_bytes : (size_t)64 << 20;
    a->flush_ms = cfg && cfg->flush_ms ? cfg->flush_ms : 100;
}

int pv_afpacket_open(const pv_afpacket_config *cfg, pv_afpacket **out)
{
    if (!cfg || !out) return fail(PV_EINVAL, "null argument");
    *out = nullptr;
    auto *a = new pv_afpacket();
    apply_defaults(cfg, a);
    const uint32_t frame_size = cfg->frame_size ? cfg->frame_size : 1u << 11;
    const std::string ifname = cfg->interface ? cfg->interface : "any";
    auto bail = [&](int rc, const char *what) {
        const int e = errno;
        delete a;
        return fail(rc, "%s: %s", what, strerror(e));
    };
    a->fd = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL)); // AFPacket::AFPacket (:41-45)
    if (a->fd == -1) return bail(errno == EPERM ? PV_EUNSUPPORTED : PV_EINVAL, "Failed to create AF_PACKET socket");
    // set_interface (:88-118)
    int ifindex = 0, iftype = 0;
    if (ifname != "any") {
        if (ifname.size() > IFNAMSIZ) {
            delete a;
            return fail(PV_EINVAL, "Invalid argument: interface name is too long: %s", ifname.c_str());
        }
        ifreq ifr{};
        strncpy(ifr.ifr_name, ifname.c_str(), sizeof(ifr.ifr_name) - 1);
        if (ioctl(a->fd, SIOCGIFINDEX, &ifr) == -1) return bail(PV_EINVAL, "Failed to get interface index from name");
        ifindex = ifr.ifr_ifindex;
        memset(&ifr, 0, sizeof ifr);
        strncpy(ifr.ifr_name, ifname.c_str(), sizeof(ifr.ifr_name) - 1);
        if (ioctl(a->fd, SIOCGIFHWADDR, &ifr) == -1) return bail(PV_EINVAL, "Failed to get interface type from name");
        iftype = ifr.ifr_hwaddr.sa_family;
    }
    (void)iftype;
    // set_socket_opts (:120-172)
    const int version = TPACKET_V3;
    if (setsockopt(a->fd, SOL_PACKET, PACKET_VERSION, &version, sizeof version) == -1)
        return bail(PV_EINVAL, "Failed to set packet v3 version on AF_PACKET socket");
    if (ifindex > 0) {
        packet_mreq mr{};
        mr.mr_type = PACKET_MR_PROMISC;
        mr.mr_ifindex = ifindex;
        if (setsockopt(a->fd, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mr, sizeof mr) == -1)
            return bail(PV_EINVAL, "Failed to enable promisc mode on AF_PACKET socket");
    }
    if (cfg->bpf_insns && cfg->bpf_len) {
        // the kernel takes a 16-bit length: validate first (at most BPF_MAXINSNS, classic-BPF rules)
        if (pv_bpf_validate(static_cast<const pv_bpf_insn *>(cfg->bpf_insns), cfg->bpf_len) != 0)
            return bail(PV_EINVAL, "invalid BPF program for the AF_PACKET socket");
        sock_fprog prog{};
        prog.len = (unsigned short)cfg->bpf_len;
        prog.filter = const_cast<sock_filter *>(static_cast<const sock_filter *>(cfg->bpf_insns));
        if (setsockopt(a->fd, SOL_SOCKET, SO_ATTACH_FILTER, &prog, sizeof prog) == -1)
            return bail(PV_EINVAL, "Failed to attach supplied BPF filter to AF_PACKET socket");
        const int lock = 1;
        if (setsockopt(a->fd, SOL_SOCKET, SO_LOCK_FILTER, &lock, sizeof lock) == -1)
            return bail(PV_EINVAL, "Failed to lock supplied BPF filter to AF_PACKET socket");
    }
    tpacket_req3 req{};
    req.tp_block_size = a->block_size;
    req.tp_frame_size = frame_size;
    req.tp_block_nr = a->num_blocks;
    req.tp_frame_nr = (a->block_size * a->num_blocks) / frame_size;
    req.tp_retire_blk_tov = 60; // ms
    req.tp_feature_req_word = TP_FT_REQ_FILL_RXHASH;
    if (setsockopt(a->fd, SOL_PACKET, PACKET_RX_RING, &req, sizeof req) == -1)
        return bail(PV_EINVAL, "Failed to enable RX_RING for AF_PACKET socket");
    // setup (:174-212)
    a->map_bytes = (size_t)a->block_size * a->num_blocks;
    void *mp = mmap(nullptr, a->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_LOCKED, a->fd, 0);
    if (mp == MAP_FAILED) return bail(PV_EINVAL, "Failed to initialize RX_RING mmap");
    a->map = static_cast<uint8_t *>(mp);
    a->own_map = true;
    sockaddr_ll sll{};
    sll.sll_family = AF_PACKET;
    sll.sll_protocol = htons(ETH_P_ALL);
    sll.sll_ifindex = ifindex;
    if (bind(a->fd, reinterpret_cast<sockaddr *>(&sll), sizeof sll) == -1)
        return bail(PV_EINVAL, "Failed binding the AF_PACKET socket to the specified interface");
    if (cfg->fanout_group_id >= 0) {
        const int arg = cfg->fanout_group_id | (PACKET_FANOUT_LB << 16);
        if (setsockopt(a->fd, SOL_PACKET, PACKET_FANOUT, &arg, sizeof arg) < 0)
            return bail(PV_EINVAL, "Failed to configure fanout for AF_PACKET socket");
    }
    a->init_staging();
    *out = a;
    return 0;
}

int pv_afpacket_attach(uint8_t *ring, uint32_t block_size, uint32_t num_blocks, int wake_fd, const pv_afpacket_config *cfg,
                       pv_afpacket **out)
{
    if (!ring || !out || block_size < sizeof(tpacket_block_desc) || !num_blocks) return fail(PV_EINVAL, "bad ring");
    auto *a = new pv_afpacket();
    apply_defaults(cfg, a);
    a->block_size = block_size;
    a->num_blocks = num_blocks;
    a->map = ring;
    a->map_bytes = (size_t)block_size * num_blocks;
    a->wake_fd = wake_fd;
    a->init_staging();
    *out = a;
    return 0;
}

// the loop of a capture whose running flag the caller has set
static int run_loop(pv_afpacket *a, pv_afpacket_sink sink, void *user)
{
    a->sink = sink;
    a->user = user;
    a->rc = 0;
    a->quit = false;
    a->worker = std::thread([a] { a->work(); });
    a->capture();
    {
        std::lock_guard<std::mutex> g(a->m);
        a->quit = true;
    }
    a->cv.notify_all();
    a->worker.join();
    a->running = false;
    std::lock_guard<std::mutex> g(a->m);
    return a->rc;
}

int pv_afpacket_run(pv_afpacket *a, pv_afpacket_sink sink, void *user)
{
    if (!a || !sink) return fail(PV_EINVAL, "null argument");
    if (a->running.exchange(true)) return fail(PV_EINVAL, "capture already running");
    return run_loop(a, sink, user);
}

int pv_afpacket_start(pv_afpacket *a, pv_ctx *ctx)
{
    if (!a || !ctx) return fail(PV_EINVAL, "null argument");
    if (a->cap_thread.joinable() || a->running.exchange(true)) return fail(PV_EINVAL, "capture already started");
    a->cap_thread = std::thread([a, ctx] { run_loop(a, sink_process_host, ctx); });
    return 0;
}

int pv_afpacket_stop(pv_afpacket *a)
{
    if (!a) return fail(PV_EINVAL, "null argument");
    a->running = false;
    if (a->cap_thread.joinable()) a->cap_thread.join();
    std::lock_guard<std::mutex> g(a->m);
    return a->rc;
}

int pv_afpacket_stats(pv_afpacket *a, pv_afpacket_counters *out)
{
    if (!a || !out) return fail(PV_EINVAL, "null argument");
    a->read_stats();
    out->blocks = a->blocks;
    out->packets = a->packets;
    out->batches = a->batches;
    out->bytes = a->bytes;
    out->kernel_packets = a->kpackets.load();
    out->kernel_drops = a->drops.load();
    out->kernel_freezes = a->freezes.load();
    return 0;
}

void pv_afpacket_close(pv_afpacket *a)
{
    if (!a) return;
    pv_afpacket_stop(a);
    delete a;
}

} // extern "C"
