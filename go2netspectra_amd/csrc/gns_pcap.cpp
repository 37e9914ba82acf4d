// gns_pcap.cpp -- pcap file -> 64-byte header records + wire lengths.
//
// Replaces the per-packet gopacket/libpcap loop of pkg/pcap/reader.go:35-49 on
// the ingest side: one sequential pass over the file, no per-packet heap
// objects; the records feed gns_cm_insert_headers / gns_ss_insert_headers,
// which parse on the GPU.  Wire length = pcap orig_len = gopacket
// Metadata().Length (internal/protocol/parser.go:30-33).
//
// Each frame becomes one record (gns_frame.cpp frame_record): frames of the
// device fast-path shape are copied verbatim (first 64 bytes), all others are
// decoded here, on the whole captured frame, into pre-parsed 0x88B5 records
// (or a record the device drops, for a frame without an IP layer), so no
// record leaves the device parser "unsupported".
//
// Supported: classic pcap (micro- and nanosecond magic, either byte order) and
// pcapng (any byte order, several sections and interfaces, if_tsresol /
// if_tsoffset), linktype Ethernet (1); other linktypes are rejected.
#include <cstdio>
#include <cstring>
#include <vector>

#include "gns_common.hpp"

namespace {

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
inline uint16_t bswap16(uint16_t x) { return __builtin_bswap16(x); }

thread_local uint64_t t_counts[3];  // verbatim, escaped, dropped of this thread's last pack

struct Sink {  // record output (the first `cap` packets) and counters
    uint8_t *hdr;
    uint32_t *wirelen;
    int64_t *ts_ns;
    uint64_t cap, written = 0, n = 0;
    uint64_t kinds[3] = {0, 0, 0};
    void emit(const uint8_t *data, uint32_t incl, uint32_t orig, int64_t ts) {
        if (written < cap && hdr && wirelen) {
            kinds[gns::frame_record(data, incl, orig, hdr + written * 64)]++;
            wirelen[written] = orig;
            if (ts_ns) ts_ns[written] = ts;
            written++;
        }
        n++;
    }
};

// classic pcap records after the 24-byte file header
int classic(FILE *f, const char *path, const uint8_t (&gh)[24], uint32_t magic, Sink &o) {
    using gns::set_error;
    const bool nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    const bool swap = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    uint32_t linktype;
    memcpy(&linktype, gh + 20, 4);
    if (swap) linktype = bswap32(linktype);
    if ((linktype & 0x0FFFFFFFu) != 1u) {
        set_error("%s: linktype %u not supported (Ethernet only)", path, linktype);
        return GNS_E_ARG;
    }
    std::vector<uint8_t> pkt(1 << 18);
    for (;;) {
        uint8_t rh[16];
        const size_t got = fread(rh, 1, 16, f);
        if (got != 16) break;  // end of file, or a truncated trailer: gopacket stops too
        uint32_t incl, orig, tsec, tfrac;
        memcpy(&tsec, rh, 4);
        memcpy(&tfrac, rh + 4, 4);
        memcpy(&incl, rh + 8, 4);
        memcpy(&orig, rh + 12, 4);
        if (swap) { incl = bswap32(incl); orig = bswap32(orig); tsec = bswap32(tsec); tfrac = bswap32(tfrac); }
        if (incl > pkt.size()) pkt.resize(incl);
        if (fread(pkt.data(), 1, incl, f) != incl) break;
        o.emit(pkt.data(), incl, orig, (int64_t)(int32_t)tsec * 1000000000ll + (int64_t)tfrac * (nsec ? 1 : 1000));
    }
    return GNS_OK;
}

// pcapng (the format libpcap's pcap_open_offline also reads, which is what
// gopacket's pcap.OpenOffline calls, reader.go:21): Section Header, Interface
// Description, Enhanced / Simple / obsolete Packet blocks; every other block
// type is skipped.  Timestamps follow the interface's if_tsresol (power of ten
// or of two, default microseconds) and if_tsoffset, scaled to nanoseconds the
// way libpcap scales them for a nanosecond-precision handle.
struct Iface {
    uint32_t snaplen;
    uint64_t units;  // timestamp units per second
    int64_t offset;  // if_tsoffset, seconds
};

inline uint64_t pow10u(uint32_t e) { uint64_t v = 1; while (e--) v *= 10; return v; }

int64_t ng_ts_ns(const Iface &ifc, uint64_t t) {
    const uint64_t sec = t / ifc.units + (uint64_t)ifc.offset;
    const uint64_t frac = t % ifc.units;
    const uint64_t ns = (uint64_t)((unsigned __int128)frac * 1000000000u / ifc.units);
    return (int64_t)(sec * 1000000000ull + ns);
}

int pcapng(FILE *f, const char *path, Sink &o) {
    using gns::set_error;
    std::vector<uint8_t> body(1 << 16);
    std::vector<Iface> ifs;
    bool swap = false, have_shb = false, first_swap = false;
    for (;;) {
        uint8_t bh[8];
        if (fread(bh, 1, 8, f) != 8) break;  // end of file (a partial block header: stop)
        uint32_t type, len;
        memcpy(&type, bh, 4);
        memcpy(&len, bh + 4, 4);
        if (type == 0x0A0D0D0Au) {  // Section Header: its byte-order magic sets the byte order
            uint32_t bom;
            if (fread(&bom, 1, 4, f) != 4) break;
            if (bom == 0x1A2B3C4Du) swap = false;
            else if (bom == 0x4D3C2B1Au) swap = true;
            else { set_error("%s: pcapng section with bad byte-order magic %08x", path, bom); return GNS_E_ARG; }
            // libpcap's pcap_open_offline (which gopacket's OpenOffline calls) reads every
            // section with the first one's byte order and rejects a file whose sections differ
            if (!have_shb) first_swap = swap;
            else if (swap != first_swap) {
                set_error("%s: pcapng sections with different byte orders", path);
                return GNS_E_ARG;
            }
            if (swap) len = bswap32(len);
            if (len < 28 || (len & 3u)) { set_error("%s: bad pcapng section header length %u", path, len); return GNS_E_ARG; }
            if (body.size() < len) body.resize(len);
            if (fread(body.data(), 1, len - 12, f) != len - 12) break;
            uint16_t major;
            memcpy(&major, body.data(), 2);
            if (swap) major = bswap16(major);
            if (major != 1) { set_error("%s: pcapng major version %u not supported", path, major); return GNS_E_ARG; }
            ifs.clear();  // interface ids are per section
            have_shb = true;
            continue;
        }
        if (!have_shb) { set_error("%s: pcapng block before the section header", path); return GNS_E_ARG; }
        if (swap) { type = bswap32(type); len = bswap32(len); }
        if (len < 12 || (len & 3u)) { set_error("%s: bad pcapng block length %u", path, len); return GNS_E_ARG; }
        const uint32_t bl = len - 12;  // body between the header and the trailing length
        if (body.size() < bl + 4) body.resize(bl + 4);
        if (fread(body.data(), 1, bl + 4, f) != bl + 4) break;  // truncated block: stop
        const uint8_t *b = body.data();
        auto u16 = [&](uint32_t off) { uint16_t v; memcpy(&v, b + off, 2); return swap ? bswap16(v) : v; };
        auto u32 = [&](uint32_t off) { uint32_t v; memcpy(&v, b + off, 4); return swap ? bswap32(v) : v; };
        if (type == 1u) {  // Interface Description
            if (bl < 8) { set_error("%s: short pcapng interface block", path); return GNS_E_ARG; }
            const uint32_t lt = u16(0);
            if (lt != 1u) { set_error("%s: linktype %u not supported (Ethernet only)", path, lt); return GNS_E_ARG; }
            Iface ifc{u32(4), 1000000ull, 0};
            for (uint32_t off = 8; off + 4 <= bl;) {
                const uint32_t code = u16(off), olen = u16(off + 2);
                if (code == 0) break;  // opt_endofopt
                if (off + 4 + olen > bl) break;
                if (code == 9 && olen >= 1) {  // if_tsresol
                    const uint8_t r = b[off + 4];
                    if (r & 0x80u) {
                        if ((r & 0x7Fu) > 63u) { set_error("%s: if_tsresol 2^-%u", path, r & 0x7Fu); return GNS_E_ARG; }
                        ifc.units = 1ull << (r & 0x7Fu);
                    } else {
                        if (r > 19u) { set_error("%s: if_tsresol 10^-%u", path, r); return GNS_E_ARG; }
                        ifc.units = pow10u(r);
                    }
                } else if (code == 14 && olen >= 8) {  // if_tsoffset
                    uint64_t v;
                    memcpy(&v, b + off + 4, 8);
                    if (swap) v = __builtin_bswap64(v);
                    ifc.offset = (int64_t)v;
                }
                off += 4 + ((olen + 3u) & ~3u);
            }
            ifs.push_back(ifc);
        } else if (type == 6u || type == 2u) {  // Enhanced Packet / obsolete Packet
            if (bl < 20) { set_error("%s: short pcapng packet block", path); return GNS_E_ARG; }
            const uint32_t id = type == 6u ? u32(0) : u16(0);
            const uint64_t t = (uint64_t)u32(4) << 32 | u32(8);
            const uint32_t incl = u32(12), orig = u32(16);
            if (id >= ifs.size()) { set_error("%s: packet on interface %u without a description block", path, id); return GNS_E_ARG; }
            if (incl > bl - 20) { set_error("%s: pcapng packet block shorter than its capture length", path); return GNS_E_ARG; }
            o.emit(b + 20, incl, orig, ng_ts_ns(ifs[id], t));
        } else if (type == 3u) {  // Simple Packet: interface 0, no timestamp
            if (bl < 4) { set_error("%s: short pcapng simple packet block", path); return GNS_E_ARG; }
            if (ifs.empty()) { set_error("%s: simple packet without an interface description block", path); return GNS_E_ARG; }
            const uint32_t orig = u32(0);
            uint32_t incl = orig;
            if (ifs[0].snaplen && incl > ifs[0].snaplen) incl = ifs[0].snaplen;
            if (incl > bl - 4) incl = bl - 4;
            o.emit(b + 4, incl, orig, 0);
        }
    }
    return GNS_OK;
}

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
    Sink o{hdr, wirelen, ts_ns, cap};
    memset(t_counts, 0, sizeof t_counts);
    int rc;
    uint8_t gh[24];
    if (fread(gh, 1, 8, f) != 8) { fclose(f); set_error("%s: short capture file header", path); return GNS_E_ARG; }
    uint32_t magic;
    memcpy(&magic, gh, 4);
    if (magic == 0x0A0D0D0Au) {
        if (fseek(f, 0, SEEK_SET) != 0) { fclose(f); set_error("%s: cannot rewind", path); return GNS_E_ARG; }
        rc = pcapng(f, path, o);
    } else if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du || magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) {
        if (fread(gh + 8, 1, 16, f) != 16) { fclose(f); set_error("%s: short pcap header", path); return GNS_E_ARG; }
        rc = classic(f, path, gh, magic, o);
    } else {
        fclose(f);
        set_error("%s: neither pcap nor pcapng (magic %08x)", path, magic);
        return GNS_E_ARG;
    }
    fclose(f);
    if (rc != GNS_OK) return rc;
    memcpy(t_counts, o.kinds, sizeof t_counts);
    if (total) *total = o.n;
    return (int64_t)o.written;
}

extern "C" int64_t gns_pack_pcap(const char *path, uint8_t *hdr, uint32_t *wirelen, uint64_t cap,
                                 uint64_t *total) {
    return gns_pack_pcap_ts(path, hdr, wirelen, nullptr, cap, total);
}

extern "C" int gns_pack_counts(uint64_t out[3]) {
    if (!out) { gns::set_error("null argument"); return GNS_E_ARG; }
    memcpy(out, t_counts, sizeof t_counts);
    return GNS_OK;
}
