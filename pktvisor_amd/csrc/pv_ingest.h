// SPDX-License-Identifier: MPL-2.0
// pv_ingest.h — host side of the pcap-record ingest: a persistent worker pool and the
// parallel record index the host-memory path (pv_process_host) runs per chunk.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/pvgpu.h"

namespace pvi {

// Fixed set of threads running parallel_for(n, f): f(0..n-1), the caller taking part.
class Pool {
public:
    explicit Pool(unsigned nthreads);
    ~Pool();
    unsigned size() const { return (unsigned)th_.size() + 1; }
    void parallel_for(unsigned n, const std::function<void(unsigned)> &f);

private:
    void run(unsigned self);
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)> *job_ = nullptr;
    unsigned n_ = 0, next_ = 0, busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Host threads for the ingest (PV_HOST_THREADS, else the online CPUs, at most 16).
unsigned default_threads();

// pv_index_records over [recs, recs + bytes) with the walk split across the pool; the
// result (offsets, sec changes, info, return code) is identical to the sequential walk.
// copy_dst (optional): the bytes are also copied there, each segment by the thread that
// walks it.
int index_records_parallel(Pool &pool, const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets,
                           uint64_t max_records, uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes,
                           pv_index_info *info, uint8_t *copy_dst = nullptr);

// memcpy split across the pool
void copy_parallel(Pool &pool, void *dst, const void *src, size_t bytes);

} // namespace pvi
