// gns_pcap.cpp -- pcap file -> 64-byte header records + wire lengths.
//
// Replaces the per-packet gopacket/libpcap loop of pkg/pcap/reader.go:35-49 on
// the ingest side: the file is mapped read-only and walked once (record
// boundaries only touch the 16-byte record headers and the first bytes of each
// frame), no per-packet heap objects; the records feed gns_cm_insert_headers /
// gns_ss_insert_headers, which parse on the GPU.  Wire length = pcap orig_len =
// gopacket Metadata().Length (internal/protocol/parser.go:30-33).
//
// The walk collects frame descriptors in slabs of 2^17; each slab's records are
// built by a few host threads (GNS_PACK_THREADS, default min(16, cores)), each
// thread a contiguous range of the slab, so the output order is the file order.
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
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <thread>
#include <vector>

#include "gns_common.hpp"

namespace {

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
inline uint16_t bswap16(uint16_t x) { return __builtin_bswap16(x); }

thread_local uint64_t t_counts[3];  // verbatim, escaped, dropped of this thread's last pack

struct Desc {
    const uint8_t *frame;
    uint32_t incl, orig;
    int64_t ts;
};

int pack_threads() {
    if (const char *e = getenv("GNS_PACK_THREADS")) {
        const int v = atoi(e);
        if (v > 0) return std::min(v, 64);
    }
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hc ? hc : 1u));
}

struct Sink {  // record output (the first `cap` packets) and counters
    uint8_t *hdr;
    uint32_t *wirelen;
    int64_t *ts_ns;
    uint64_t cap, written = 0, n = 0;
    uint64_t kinds[3] = {0, 0, 0};
    // compact mode (gns_pack_pcap_compact): 16-byte records into rec16, the
    // records that do not fit into side64 (side_cap of them; side_need counts all)
    uint8_t *rec16 = nullptr, *side64 = nullptr;
    uint64_t side_cap = 0, side_need = 0;
    bool rec_len = false;                // the 16-byte form (wire lengths inside the records)
    std::atomic<uint64_t> too_long{0};   // its frames with a wire length above 65535
    std::vector<Desc> slab;
    int nthreads = 1;
    static constexpr size_t kSlab = 1u << 17;
    bool out_ok() const { return (hdr || rec16) && (wirelen || rec_len); }
    void emit(const uint8_t *data, uint32_t incl, uint32_t orig, int64_t ts) {
        n++;
        if (written + slab.size() >= cap || !out_ok()) return;
        slab.push_back(Desc{data, incl, orig, ts});
        if (slab.size() == kSlab) flush();
    }
    void flush() {  // build the slab's records (file order)
        build(slab.data(), slab.size());
        slab.clear();
    }
    // a walked piece of the capture, in file order (no emit/slab copy): counted, and
    // its records built up to cap
    void take(const std::vector<Desc> &v) {
        flush();
        n += v.size();
        if (!out_ok() || written >= cap) return;
        build(v.data(), (size_t)std::min<uint64_t>(v.size(), cap - written));
    }
    void build(const Desc *src, size_t m) {  // records of src[0, m), several threads over contiguous ranges
        if (!m) return;
        const int T = (int)std::min<size_t>((size_t)nthreads, (m + 4095) / 4096);
        uint64_t part[64][3] = {};
        std::vector<std::vector<uint8_t>> side(T);   // per thread: its side records, in order
        std::vector<std::vector<uint64_t>> at(T);    // and the packets that name them
        auto work = [&](int t) {
            const size_t i0 = m * t / T, i1 = m * (t + 1) / T;
            uint8_t tmp[64];
            for (size_t i = i0; i < i1; i++) {
                const Desc &dsc = src[i];
                const uint64_t j = written + i;
                uint8_t *r = rec16 ? tmp : hdr + j * 64;
                const int code = gns::frame_record(dsc.frame, dsc.incl, dsc.orig, r);
                part[t][code]++;
                int cls = -2;
                if (rec16 && rec_len) {
                    cls = gns::compact_record16(code, r, dsc.orig, rec16 + j * 16);
                    if (cls < 0) too_long++;
                } else if (rec16) {
                    cls = gns::compact_record(code, r, rec16 + j * 16);
                }
                if (cls == gns::kRecSide) {
                    side[t].insert(side[t].end(), r, r + 64);
                    at[t].push_back(j);
                }
                if (wirelen) wirelen[j] = dsc.orig;
                if (ts_ns) ts_ns[j] = dsc.ts;
            }
        };
        if (T <= 1) {
            work(0);
        } else {
            std::vector<std::thread> th;
            th.reserve(T - 1);
            for (int t = 1; t < T; t++) th.emplace_back(work, t);
            work(0);
            for (auto &x : th) x.join();
        }
        for (int t = 0; t < T; t++) {
            for (int k = 0; k < 3; k++) kinds[k] += part[t][k];
            for (size_t q = 0; q < at[t].size(); q++) {  // side indices in file order
                const uint64_t idx = side_need++;
                const uint32_t w0 = (uint32_t)idx;
                memcpy(rec16 + at[t][q] * 16, &w0, 4);
                if (idx < side_cap && side64) memcpy(side64 + idx * 64, side[t].data() + q * 64, 64);
            }
        }
        written += m;
    }
};

// The capture as one read-only byte range (mapped; read into memory when the
// file cannot be mapped), consumed front to back.
struct Cursor {
    const uint8_t *p = nullptr;
    size_t n = 0, off = 0;
    // the next k bytes, or null at a (truncated) end
    const uint8_t *take(size_t k) {
        if (k > n - off) return nullptr;
        const uint8_t *r = p + off;
        off += k;
        return r;
    }
};

// classic pcap records after the 24-byte file header
// One classic-pcap record header at off: (incl, orig, ts), or false past the end.
struct RecHdr {
    uint32_t incl, orig;
    int64_t ts;
};
inline bool rec_at(const uint8_t *p, size_t n, size_t off, bool swap, bool nsec, RecHdr &h) {
    if (off + 16 > n) return false;
    uint32_t tsec, tfrac;
    memcpy(&tsec, p + off, 4);
    memcpy(&tfrac, p + off + 4, 4);
    memcpy(&h.incl, p + off + 8, 4);
    memcpy(&h.orig, p + off + 12, 4);
    if (swap) { h.incl = bswap32(h.incl); h.orig = bswap32(h.orig); tsec = bswap32(tsec); tfrac = bswap32(tfrac); }
    h.ts = (int64_t)(int32_t)tsec * 1000000000ll + (int64_t)tfrac * (nsec ? 1 : 1000);
    return true;
}

// The record walk is a chain through the file (each header gives the next one's offset), so
// one thread walking a large capture is bound by its memory latency.  Large captures are
// walked in parallel: the file is cut into one piece per thread, each piece after the first
// starts at the first offset whose header and the next three chain plausibly (incl <= the
// snap length, orig >= incl, ...), and each thread walks until it reaches its successor's
// start.  The pieces are used only if every walk lands exactly on the next piece's start --
// then their records are the sequential walk's, in the same order; otherwise the capture is
// walked sequentially.
struct PieceWalk {
    std::vector<Desc> d;
    size_t end = 0;  // offset where the walk stopped
    bool stopped = false;  // a truncated record or the file's end
};

inline bool plausible(const uint8_t *p, size_t n, size_t off, bool swap, bool nsec, uint32_t snap) {
    for (int k = 0; k < 4; k++) {
        RecHdr h;
        if (!rec_at(p, n, off, swap, nsec, h)) return k > 0;  // a chain reaching the end is fine
        if (h.incl > snap || h.incl < 14 || h.orig < h.incl || h.orig > (1u << 24)) return false;
        off += 16 + (size_t)h.incl;
        if (off > n) return k > 0;
    }
    return true;
}

int classic(Cursor &f, const char *path, const uint8_t *gh, uint32_t magic, Sink &o) {
    using gns::set_error;
    const bool nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    const bool swap = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    uint32_t linktype, snap;
    memcpy(&linktype, gh + 20, 4);
    memcpy(&snap, gh + 16, 4);
    if (swap) { linktype = bswap32(linktype); snap = bswap32(snap); }
    if ((linktype & 0x0FFFFFFFu) != 1u) {
        set_error("%s: linktype %u not supported (Ethernet only)", path, linktype);
        return GNS_E_ARG;
    }
    if (snap == 0 || snap > (1u << 24)) snap = 1u << 24;
    const int T = o.nthreads;
    const size_t n = f.n, base = f.off;
    size_t par_min = (size_t)64 << 20;  // below this the walk is short anyway
    if (const char *e = getenv("GNS_PACK_PAR_MIN")) par_min = (size_t)strtoull(e, nullptr, 10);
    // windows of the file (1 GiB by default) bound the descriptors held at once; each window
    // starts where the previous one's last piece stopped, a record start by the same induction
    size_t win = (size_t)1 << 30;
    if (const char *e = getenv("GNS_PACK_WINDOW")) win = std::max<size_t>(4096, (size_t)strtoull(e, nullptr, 10));
    if (T > 1 && n - base >= par_min && o.out_ok()) {
        size_t pos = base;
        std::vector<PieceWalk> w(T);
        while (pos < n) {
            const size_t wend = std::min(n, pos + win);  // the window: records starting before wend
            std::vector<size_t> start(T + 1, wend);
            start[0] = pos;
            bool ok = true;
            for (int t = 1; t < T && ok; t++) {
                size_t off = pos + (wend - pos) * (size_t)t / (size_t)T;
                const size_t lim = std::min(wend, off + ((size_t)1 << 20));  // a record is far shorter
                while (off < lim && !plausible(f.p, n, off, swap, nsec, snap)) off++;
                if (off >= lim || off <= start[t - 1]) ok = false;
                start[t] = off;
            }
            if (!ok) break;  // the rest sequentially, from pos
            auto walk = [&](int t) {
                size_t off = start[t];
                const size_t stop = start[t + 1];
                PieceWalk &pw = w[t];
                pw.d.clear();
                pw.stopped = false;
                pw.d.reserve((stop - off) / 64 + 16);
                while (off < stop) {
                    if (off + 4096 < n) {
                        __builtin_prefetch(f.p + off + 2048);
                        __builtin_prefetch(f.p + off + 4096);
                    }
                    RecHdr h;
                    if (!rec_at(f.p, n, off, swap, nsec, h) || off + 16 + (size_t)h.incl > n) {
                        pw.stopped = true;  // end of file, or a truncated trailer: gopacket stops too
                        break;
                    }
                    pw.d.push_back(Desc{f.p + off + 16, h.incl, h.orig, h.ts});
                    off += 16 + (size_t)h.incl;
                }
                pw.end = off;
            };
            std::vector<std::thread> th;
            th.reserve(T - 1);
            for (int t = 1; t < T; t++) th.emplace_back(walk, t);
            walk(0);
            for (auto &x : th) x.join();
            for (int t = 0; t + 1 < T && ok; t++) ok = !w[t].stopped && w[t].end == start[t + 1];
            if (!ok) break;  // the rest sequentially, from pos
            for (int t = 0; t < T; t++) o.take(w[t].d);
            if (w[T - 1].stopped) return GNS_OK;
            pos = w[T - 1].end;
        }
        f.off = pos;  // a record start (or the end of the file)
    }
    for (;;) {
        // the walk is a chain through the file (each header gives the next one's offset):
        // touch the lines a few KB ahead so the next headers are in cache when reached
        if (f.off + 4096 < f.n) {
            __builtin_prefetch(f.p + f.off + 2048);
            __builtin_prefetch(f.p + f.off + 4096);
        }
        const uint8_t *rh = f.take(16);
        if (!rh) break;  // end of file, or a truncated trailer: gopacket stops too
        uint32_t incl, orig, tsec, tfrac;
        memcpy(&tsec, rh, 4);
        memcpy(&tfrac, rh + 4, 4);
        memcpy(&incl, rh + 8, 4);
        memcpy(&orig, rh + 12, 4);
        if (swap) { incl = bswap32(incl); orig = bswap32(orig); tsec = bswap32(tsec); tfrac = bswap32(tfrac); }
        const uint8_t *pkt = f.take(incl);
        if (!pkt) break;
        o.emit(pkt, incl, orig, (int64_t)(int32_t)tsec * 1000000000ll + (int64_t)tfrac * (nsec ? 1 : 1000));
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

int pcapng(Cursor &f, const char *path, Sink &o) {
    using gns::set_error;
    std::vector<Iface> ifs;
    bool swap = false, have_shb = false, first_swap = false;
    for (;;) {
        const uint8_t *bh = f.take(8);
        if (!bh) break;  // end of file (a partial block header: stop)
        uint32_t type, len;
        memcpy(&type, bh, 4);
        memcpy(&len, bh + 4, 4);
        if (type == 0x0A0D0D0Au) {  // Section Header: its byte-order magic sets the byte order
            const uint8_t *bp = f.take(4);
            if (!bp) break;
            uint32_t bom;
            memcpy(&bom, bp, 4);
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
            const uint8_t *sb = f.take(len - 12);
            if (!sb) break;
            uint16_t major;
            memcpy(&major, sb, 2);
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
        const uint8_t *b = f.take((size_t)bl + 4);
        if (!b) break;  // truncated block: stop
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

// The capture file, mapped read-only (or read whole when it cannot be mapped).
struct Capture {
    int fd = -1;
    void *map = nullptr;
    size_t size = 0;
    std::vector<uint8_t> copy;
    const uint8_t *data() const { return map ? static_cast<const uint8_t *>(map) : copy.data(); }
    int open_file(const char *path) {
        fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) { gns::set_error("cannot open %s", path); return GNS_E_ARG; }
        struct stat st;
        if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
            size = (size_t)st.st_size;
            map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
            if (map == MAP_FAILED) map = nullptr;
            else (void)madvise(map, size, MADV_SEQUENTIAL);
        }
        if (!map) {  // not mappable (a pipe, /dev/stdin ...): read it whole
            copy.clear();
            uint8_t buf[1 << 16];
            for (;;) {
                const ssize_t r = ::read(fd, buf, sizeof buf);
                if (r < 0) { gns::set_error("cannot read %s", path); return GNS_E_ARG; }
                if (r == 0) break;
                copy.insert(copy.end(), buf, buf + r);
            }
            size = copy.size();
        }
        return GNS_OK;
    }
    ~Capture() {
        if (map) munmap(map, size);
        if (fd >= 0) ::close(fd);
    }
};

}  // namespace

namespace {

int64_t pack(const char *path, Sink &o, uint64_t *total) {
    using gns::set_error;
    if (!path) { set_error("null path"); return GNS_E_ARG; }
    Capture cf;
    GNS_TRY(cf.open_file(path));
    Cursor f{cf.data(), cf.size, 0};
    o.nthreads = pack_threads();
    if (o.cap && o.out_ok()) o.slab.reserve(std::min<uint64_t>(o.cap, Sink::kSlab));
    memset(t_counts, 0, sizeof t_counts);
    int rc;
    const uint8_t *gh = f.take(8);
    if (!gh) { set_error("%s: short capture file header", path); return GNS_E_ARG; }
    uint32_t magic;
    memcpy(&magic, gh, 4);
    if (magic == 0x0A0D0D0Au) {
        f.off = 0;
        rc = pcapng(f, path, o);
    } else if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du || magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) {
        if (!f.take(16)) { set_error("%s: short pcap header", path); return GNS_E_ARG; }
        rc = classic(f, path, gh, magic, o);
    } else {
        set_error("%s: neither pcap nor pcapng (magic %08x)", path, magic);
        return GNS_E_ARG;
    }
    if (rc != GNS_OK) return rc;
    o.flush();
    memcpy(t_counts, o.kinds, sizeof t_counts);
    if (total) *total = o.n;
    return (int64_t)o.written;
}

}  // namespace

// ts_ns: capture timestamps in ns (gopacket's pcap handle opens files with
// nanosecond precision: usec files scale by 1000, nsec files as recorded).
extern "C" int64_t gns_pack_pcap_ts(const char *path, uint8_t *hdr, uint32_t *wirelen, int64_t *ts_ns,
                                    uint64_t cap, uint64_t *total) {
    Sink o{hdr, wirelen, ts_ns, cap};
    return pack(path, o, total);
}

// compact records (IN_REC16) for the PCIe-bound host path: 16 bytes + the wire
// length per packet, the frames whose tuple is not an IPv4 one as 64-byte side
// records (GNS_E_RANGE when side_cap is too small: *n_side = the number needed)
extern "C" int64_t gns_pack_pcap_compact(const char *path, uint8_t *rec16, uint32_t *wirelen, uint64_t cap,
                                         uint8_t *side64, uint64_t side_cap, uint64_t *n_side, uint64_t *total) {
    Sink o{nullptr, wirelen, nullptr, cap};
    o.rec16 = rec16;
    o.side64 = side64;
    o.side_cap = side_cap;
    const int64_t r = pack(path, o, total);
    if (n_side) *n_side = o.side_need;
    if (r >= 0 && o.side_need > side_cap) {
        gns::set_error("%s: %llu side records needed, room for %llu", path, (unsigned long long)o.side_need,
                       (unsigned long long)side_cap);
        return GNS_E_RANGE;
    }
    return r;
}

// the 16-byte form (gns_cm_insert_compact with no wirelen array): the wire length rides in
// each record; GNS_E_RANGE when a frame's wire length exceeds 65535
extern "C" int64_t gns_pack_pcap_compact16(const char *path, uint8_t *rec16, uint64_t cap, uint8_t *side64,
                                           uint64_t side_cap, uint64_t *n_side, uint64_t *total) {
    Sink o{nullptr, nullptr, nullptr, cap};
    o.rec16 = rec16;
    o.rec_len = true;
    o.side64 = side64;
    o.side_cap = side_cap;
    const int64_t r = pack(path, o, total);
    if (n_side) *n_side = o.side_need;
    if (r >= 0 && o.too_long.load()) {
        gns::set_error("%s: %llu frames with a wire length above 65535 (use the 20-byte form)", path,
                       (unsigned long long)o.too_long.load());
        return GNS_E_RANGE;
    }
    if (r >= 0 && o.side_need > side_cap) {
        gns::set_error("%s: %llu side records needed, room for %llu", path, (unsigned long long)o.side_need,
                       (unsigned long long)side_cap);
        return GNS_E_RANGE;
    }
    return r;
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
