// Host-code sanitizer driver (tests/test_frames.py::test_host_decoders_under_sanitizers).
// Built by the test from go2netspectra_amd/csrc/gns_frame.cpp and gns_pcap.cpp with
// AddressSanitizer + UndefinedBehaviorSanitizer (host code only, --cuda-host-only):
//   frames IN OUT   IN = records {u32 caplen, u32 wirelen, caplen bytes}; each frame is
//                   copied into a heap block of exactly caplen bytes, so a read past the
//                   captured bytes is reported.  OUT = per frame rc (1 B), the 64-B record,
//                   the compact class (1 B) and the 16-B compact record.
//   pcap FILE...    packs each capture in both forms (64-B records, compact records with
//                   their side array) and prints "<n> <n_compact> <n_side>" per file.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace gns {
void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    va_end(ap);
}
int compact_record(int code, const uint8_t *rec, uint8_t *out16);
}  // namespace gns

extern "C" int gns_frame_record(const uint8_t *frame, uint32_t caplen, uint32_t wirelen, uint8_t *rec64);
extern "C" int64_t gns_pack_pcap(const char *path, uint8_t *hdr, uint32_t *wirelen, uint64_t cap, uint64_t *total);
extern "C" int64_t gns_pack_pcap_compact(const char *path, uint8_t *rec16, uint32_t *wirelen, uint64_t cap,
                                         uint8_t *side64, uint64_t side_cap, uint64_t *n_side, uint64_t *total);

static int run_frames(const char *in, const char *out) {
    FILE *f = fopen(in, "rb");
    FILE *o = fopen(out, "wb");
    if (!f || !o) return 3;
    uint32_t h[2];
    while (fread(h, 4, 2, f) == 2) {
        uint8_t *frame = static_cast<uint8_t *>(malloc(h[0] ? h[0] : 1));
        if (h[0] && fread(frame, 1, h[0], f) != h[0]) return 4;
        uint8_t rec[64], c16[16];
        const int rc = gns_frame_record(frame, h[0], h[1], rec);
        free(frame);
        const int cls = gns::compact_record(rc, rec, c16);
        const uint8_t b0 = (uint8_t)rc, b1 = (uint8_t)cls;
        fwrite(&b0, 1, 1, o);
        fwrite(rec, 1, 64, o);
        fwrite(&b1, 1, 1, o);
        fwrite(c16, 1, 16, o);
    }
    fclose(f);
    fclose(o);
    return 0;
}

static int run_pcap(int argc, char **argv) {
    const uint64_t cap = 1 << 16;
    std::vector<uint8_t> hdr(cap * 64), rec16(cap * 16), side(cap * 64);
    std::vector<uint32_t> wl(cap);
    for (int i = 0; i < argc; i++) {
        uint64_t total = 0, total2 = 0, n_side = 0;
        const int64_t n = gns_pack_pcap(argv[i], hdr.data(), wl.data(), cap, &total);
        const int64_t n2 = gns_pack_pcap_compact(argv[i], rec16.data(), wl.data(), cap, side.data(), cap, &n_side, &total2);
        printf("%lld %lld %llu\n", (long long)n, (long long)n2, (unsigned long long)n_side);
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 4 && !strcmp(argv[1], "frames")) return run_frames(argv[2], argv[3]);
    if (argc >= 3 && !strcmp(argv[1], "pcap")) return run_pcap(argc - 2, argv + 2);
    fprintf(stderr, "usage: frames IN OUT | pcap FILE...\n");
    return 2;
}
