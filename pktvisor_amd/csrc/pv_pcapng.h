// SPDX-License-Identifier: MPL-2.0
// pcapng capture files into classic pcap records (pv_pcapng.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace pvi {

enum { PVNG_EFORMAT = -2, PVNG_ELINKTYPES = -7 };

// pcapng bytes -> records (16-B header: ts_sec, ts_nsec, caplen, len; then the frame) appended
// to *out (NULL: count only); *linktype = the interfaces' shared linktype.
int pcapng_to_records(const uint8_t *buf, size_t bytes, std::vector<uint8_t> *out, uint32_t *linktype,
                      uint64_t *n_records);

} // namespace pvi
