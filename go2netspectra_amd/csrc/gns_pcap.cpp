// gns_pcap.cpp -- pcap file -> 64-byte header records + wire lengths.
//
// Replaces the per-packet gopacket/libpcap loop of pkg/pcap/reader.go:35-49 on
// the ingest side: one sequential pass over the file, no per-packet heap
// objects; the records feed gns_cm_insert_headers / gns_ss_insert_headers,
// which parse on the GPU.  Wire length = pcap orig_len = gopacket
// Metadata().Length (internal/protocol/parser.go:30-33).
//
// Supported: classic pcap (micro- and nanosecond magic, either byte order),
// linktype Ethernet (1).  pcapng and other linktypes are rejected.
#include <cstdio>
#include <cstring>
#include <vector>

#include "gns_common.hpp"

namespace {

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

}  // namespace

// ts_ns: capture timestamps in ns (gopacket's pcap handle opens files with
// nanosecond precision: usec files scale by 1000, nsec files as recorded).
extern "C" int64_t gns_pack_pcap_ts(const char *path, uint8_t *hdr, uint32_t *wirelen, int64_t *ts_ns,
                                    uint64_t cap, uint64_t *total) {
    using gns::set_error;
    if (!path) { set_error("null path"); return GNS_E_ARG; }
    FILE *f = fopen(path, "rb");
    if (!f) { set_error("cannot open %s", path); return GNS_E_ARG; }
    std::vector<char> iobuf(1 << 22);
    setvbuf(f, iobuf.data(), _IOFBF, iobuf.size());
    uint8_t gh[24];
    if (fread(gh, 1, 24, f) != 24) { fclose(f); set_error("%s: short pcap header", path); return GNS_E_ARG; }
    uint32_t magic;
    memcpy(&magic, gh, 4);
    bool swap = false;
    const bool nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du) swap = false;
    else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) swap = true;
    else { fclose(f); set_error("%s: not a classic pcap file (magic %08x)", path, magic); return GNS_E_ARG; }
    uint32_t linktype;
    memcpy(&linktype, gh + 20, 4);
    if (swap) linktype = bswap32(linktype);
    if ((linktype & 0x0FFFFFFFu) != 1u) {
        fclose(f);
        set_error("%s: linktype %u not supported (Ethernet only)", path, linktype);
        return GNS_E_ARG;
    }
    uint64_t n = 0, written = 0;
    std::vector<uint8_t> pkt(1 << 18);
    for (;;) {
        uint8_t rh[16];
        const size_t got = fread(rh, 1, 16, f);
        if (got == 0) break;
        if (got != 16) break;  // truncated trailer: gopacket stops too
        uint32_t incl, orig, tsec, tfrac;
        memcpy(&tsec, rh, 4);
        memcpy(&tfrac, rh + 4, 4);
        memcpy(&incl, rh + 8, 4);
        memcpy(&orig, rh + 12, 4);
        if (swap) { incl = bswap32(incl); orig = bswap32(orig); tsec = bswap32(tsec); tfrac = bswap32(tfrac); }
        if (incl > pkt.size()) pkt.resize(incl);
        if (fread(pkt.data(), 1, incl, f) != incl) break;
        if (written < cap && hdr && wirelen) {
            uint8_t *r = hdr + written * 64;
            const uint32_t c = incl < 64 ? incl : 64;
            memcpy(r, pkt.data(), c);
            if (c < 64) memset(r + c, 0, 64 - c);
            wirelen[written] = orig;
            if (ts_ns) ts_ns[written] = (int64_t)(int32_t)tsec * 1000000000ll + (int64_t)tfrac * (nsec ? 1 : 1000);
            written++;
        }
        n++;
    }
    fclose(f);
    if (total) *total = n;
    return (int64_t)written;
}

extern "C" int64_t gns_pack_pcap(const char *path, uint8_t *hdr, uint32_t *wirelen, uint64_t cap,
                                 uint64_t *total) {
    return gns_pack_pcap_ts(path, hdr, wirelen, nullptr, cap, total);
}
