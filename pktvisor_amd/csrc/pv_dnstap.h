// SPDX-License-Identifier: MPL-2.0
// dnstap input decoding (pv_dnstap.cpp): the fields of dnstap.Message the Net and DNS
// handlers read (src/inputs/dnstap/pb/dnstap.proto:229-287).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace pvi {

struct DtMessage {
    uint32_t type = 0;                 // Message.Type (1 AUTH_QUERY .. 14 UPDATE_RESPONSE)
    uint32_t family = 0, protocol = 0; // SocketFamily (1 INET, 2 INET6), SocketProtocol (1 UDP, 2 TCP, ...)
    bool has_family = false, has_protocol = false;
    std::vector<uint8_t> qaddr, raddr;
    bool has_qaddr = false, has_raddr = false;
    uint32_t qport = 0;
    bool has_qport = false;
    uint64_t qsec = 0, rsec = 0;
    uint32_t qnsec = 0, rnsec = 0;
    bool has_qsec = false, has_rsec = false;
    const uint8_t *qmsg = nullptr, *rmsg = nullptr; // into the decoded buffer
    size_t qmsg_len = 0, rmsg_len = 0;
    bool has_qmsg = false, has_rmsg = false;
    uint32_t frame_len = 0;            // the data frame's length (the handlers' `size`)
};

// Frame Streams bytes -> the dnstap MESSAGE events in stream order (frames that do not parse,
// are not MESSAGE or have no message are skipped, as DnstapInputStream skips them).
// *frames = data frames read.
int dnstap_decode(const uint8_t *buf, size_t bytes, std::vector<DtMessage> &out, uint32_t *frames);

} // namespace pvi
