#define _GNU_SOURCE
/*
 * gns_oracle_exact.c -- CPU ORACLE (test infrastructure, never product code)
 * for the exact aggregator, internal/engine/impl/exact/task.go.
 *
 * Restated the way the reference computes it: the flow key is the STRING
 * strings.Join(parts, "-") of the configured fields (generateKeyAndFields,
 * task.go:330-366), IPs printed by Go's net.IP.String() (IPv4 and IPv4-mapped
 * IPv6 as dotted quad, other IPv6 in RFC 5952 form via netip), ports and the
 * protocol in decimal.  Flows live in a string-keyed hash map (the reference's
 * sharded map[string]*Flow; sharding does not change the result):
 *   new flow:  StartTime = EndTime = ts, PacketCount = 1, ByteCount = Length
 *   existing:  EndTime = ts, PacketCount++, ByteCount += Length   (task.go:124-149)
 * Query (task.go:298-326) rebuilds the key from an encoded flow whose IP
 * fields are read as 16-byte net.IPs, and returns PacketCount<<32 | ByteCount.
 * The engine keys flows by canonical bytes instead; this oracle shares no code
 * with that path.
 */
#include "gns_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    char *key;        /* NUL-terminated Go key string */
    int64_t start, end;
    uint64_t pkts, bytes;
    uint64_t order;   /* creation order */
} ex_flow;

struct or_ex {
    uint8_t fields[8];
    uint32_t nfields;
    ex_flow *tab;     /* open addressing */
    uint64_t cap, n;
};

static uint64_t fnv1a(const char *s) {
    uint64_t h = 1469598103934665603ull;
    for (; *s; s++) { h ^= (uint8_t)*s; h *= 1099511628211ull; }
    return h;
}

/* net.IP(b).String() for len 4 or 16 (net/ip.go; netip.Addr.string6) */
static int go_ip_string(const uint8_t *b, int len, char *out) {
    if (len == 4)
        return sprintf(out, "%u.%u.%u.%u", b[0], b[1], b[2], b[3]);
    static const uint8_t mapped[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
    if (memcmp(b, mapped, 12) == 0)
        return sprintf(out, "%u.%u.%u.%u", b[12], b[13], b[14], b[15]);
    uint16_t g[8];
    for (int i = 0; i < 8; i++) g[i] = (uint16_t)(b[2 * i] << 8 | b[2 * i + 1]);
    int zs = 255, ze = 255; /* longest run (>= 2) of zero groups, first wins */
    for (int i = 0; i < 8; i++) {
        int j = i;
        while (j < 8 && g[j] == 0) j++;
        int l = j - i;
        if (l >= 2 && l > ze - zs) { zs = i; ze = j; }
    }
    int o = 0;
    for (int i = 0; i < 8; i++) {
        if (i == zs) {
            out[o++] = ':'; out[o++] = ':';
            i = ze;
            if (i >= 8) break;
        } else if (i > 0) {
            out[o++] = ':';
        }
        o += sprintf(out + o, "%x", g[i]);
    }
    out[o] = 0;
    return o;
}

or_ex *or_ex_new(const uint8_t *fields, uint32_t nfields) {
    or_ex *ex = (or_ex *)calloc(1, sizeof(or_ex));
    ex->nfields = nfields > 8 ? 8 : nfields;
    memcpy(ex->fields, fields, ex->nfields);
    ex->cap = 1024;
    ex->tab = (ex_flow *)calloc(ex->cap, sizeof(ex_flow));
    return ex;
}

void or_ex_reset(or_ex *ex) {
    for (uint64_t i = 0; i < ex->cap; i++) free(ex->tab[i].key);
    memset(ex->tab, 0, ex->cap * sizeof(ex_flow));
    ex->n = 0;
}

void or_ex_free(or_ex *ex) {
    if (!ex) return;
    or_ex_reset(ex);
    free(ex->tab);
    free(ex);
}

static ex_flow *ex_find(or_ex *ex, const char *key, int create) {
    if (create && 2 * (ex->n + 1) > ex->cap) {
        uint64_t nc = ex->cap * 2;
        ex_flow *nt = (ex_flow *)calloc(nc, sizeof(ex_flow));
        for (uint64_t i = 0; i < ex->cap; i++) {
            if (!ex->tab[i].key) continue;
            uint64_t s = fnv1a(ex->tab[i].key) & (nc - 1);
            while (nt[s].key) s = (s + 1) & (nc - 1);
            nt[s] = ex->tab[i];
        }
        free(ex->tab);
        ex->tab = nt;
        ex->cap = nc;
    }
    uint64_t s = fnv1a(key) & (ex->cap - 1);
    while (ex->tab[s].key) {
        if (strcmp(ex->tab[s].key, key) == 0) return &ex->tab[s];
        s = (s + 1) & (ex->cap - 1);
    }
    if (!create) return NULL;
    ex->tab[s].key = strdup(key);
    ex->tab[s].order = ex->n++;
    return &ex->tab[s];
}

/* generateKeyAndFields (task.go:330-366).  ipver 4: IPs are the first 4 bytes
 * of the slots (net.IP of length 4, as gopacket's IPv4 layer yields);
 * 6: 16-byte net.IPs. */
static void ex_key_tuple(const or_ex *ex, const or_tuple *t, char *out) {
    int o = 0;
    for (uint32_t i = 0; i < ex->nfields; i++) {
        if (i) out[o++] = '-';
        switch (ex->fields[i]) {
        case OR_F_SRCIP: o += go_ip_string(t->src, t->ipver == 4 ? 4 : 16, out + o); break;
        case OR_F_DSTIP: o += go_ip_string(t->dst, t->dst_ipver == 4 ? 4 : 16, out + o); break;
        case OR_F_SRCPORT: o += sprintf(out + o, "%u", t->sport); break;
        case OR_F_DSTPORT: o += sprintf(out + o, "%u", t->dport); break;
        case OR_F_PROTO: o += sprintf(out + o, "%u", t->proto); break;
        default: break;
        }
    }
    out[o] = 0;
}

/* ProcessPacket (task.go:124-149) */
void or_ex_insert(or_ex *ex, const or_tuple *t, int64_t ts, uint64_t length) {
    char key[256];
    ex_key_tuple(ex, t, key);
    ex_flow *f = ex_find(ex, key, 1);
    if (f->pkts == 0) {
        f->start = ts; f->end = ts; f->pkts = 1; f->bytes = length;
    } else {
        f->end = ts; f->pkts++; f->bytes += length;
    }
}

/* batch of PacketInfo (SoA, slots as EncodeFlow lays them out) */
void or_ex_insert_tuples(or_ex *ex, const uint8_t *src16, const uint8_t *dst16, const uint16_t *sport,
                         const uint16_t *dport, const uint8_t *proto, const uint8_t *ipver,
                         const uint32_t *length, const int64_t *ts, uint64_t n) {
    for (uint64_t p = 0; p < n; p++) {
        or_tuple t;
        memcpy(t.src, src16 + 16 * p, 16);
        memcpy(t.dst, dst16 + 16 * p, 16);
        t.sport = sport[p]; t.dport = dport[p]; t.proto = proto[p]; t.ipver = t.dst_ipver = ipver[p];
        or_ex_insert(ex, &t, ts[p], length[p]);
    }
}

/* pcap path: records parsed like parser.go; returns records inserted */
uint64_t or_ex_insert_hdr64(or_ex *ex, const uint8_t *hdr, const uint32_t *wirelen, const int64_t *ts,
                            uint64_t n) {
    uint64_t done = 0;
    for (uint64_t p = 0; p < n; p++) {
        or_tuple t;
        if (or_parse_hdr64_len(hdr + 64 * p, wirelen[p], &t) != OR_PARSE_OK) continue;
        if (t.ipver == 0 || t.dst_ipver == 0) continue; /* "?hex" keys: outside this build's scope */
        or_ex_insert(ex, &t, ts[p], wirelen[p]);
        done++;
    }
    return done;
}

/* Query (task.go:298-326): IP fields of the encoded flow are 16-byte net.IPs */
uint64_t or_ex_query(const or_ex *ex, const uint8_t *flow) {
    char key[256];
    int o = 0, off = 0;
    for (uint32_t i = 0; i < ex->nfields; i++) {
        if (i) key[o++] = '-';
        switch (ex->fields[i]) {
        case OR_F_SRCIP: case OR_F_DSTIP: o += go_ip_string(flow + off, 16, key + o); off += 16; break;
        case OR_F_SRCPORT: case OR_F_DSTPORT:
            o += sprintf(key + o, "%u", (unsigned)(flow[off] << 8 | flow[off + 1])); off += 2; break;
        case OR_F_PROTO: o += sprintf(key + o, "%u", flow[off]); off += 1; break;
        default: return 0;
        }
    }
    key[o] = 0;
    ex_flow *f = ex_find((or_ex *)ex, key, 0);
    return f ? (f->pkts << 32 | f->bytes) : 0;
}

uint64_t or_ex_count(const or_ex *ex) { return ex->n; }

/* Snapshot in creation order: keys joined by '\n' into keys_out (cap bytes),
 * counters into the arrays.  Returns the number of flows. */
uint64_t or_ex_export(const or_ex *ex, char *keys_out, uint64_t keys_cap, int64_t *start, int64_t *end,
                      uint64_t *pkts, uint64_t *bytes) {
    ex_flow **ord = (ex_flow **)calloc(ex->n ? ex->n : 1, sizeof(ex_flow *));
    for (uint64_t i = 0; i < ex->cap; i++)
        if (ex->tab[i].key) ord[ex->tab[i].order] = &ex->tab[i];
    uint64_t o = 0;
    for (uint64_t i = 0; i < ex->n; i++) {
        const ex_flow *f = ord[i];
        if (start) start[i] = f->start;
        if (end) end[i] = f->end;
        if (pkts) pkts[i] = f->pkts;
        if (bytes) bytes[i] = f->bytes;
        if (keys_out) {
            uint64_t l = strlen(f->key);
            if (o + l + 1 < keys_cap) {
                memcpy(keys_out + o, f->key, l);
                keys_out[o + l] = '\n';
                o += l + 1;
            }
        }
    }
    if (keys_out && o < keys_cap) keys_out[o] = 0;
    free(ord);
    return ex->n;
}
