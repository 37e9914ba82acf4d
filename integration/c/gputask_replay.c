/*
 * gputask_replay.c -- a C caller of libgns_sketch.so that replays, call for call,
 * what integration/go/sketchgpu/task.go's GPUTask does on its device handle
 * (the Go package cannot be compiled here: no Go toolchain).  Built against
 * include/gns_sketch.h only, linked to the shipped library:
 *
 *   NewGPUTask          -> gns_cm_create / gns_ss_create with seeds = NULL (the
 *                          engine's default row seeds), max_flows 0, device 0
 *   ProcessPacket x B   -> one gns_{cm,ss}_insert_tuples(GNS_MEM_HOST) per full
 *                          batch of BatchPackets packets (SoA host buffers)
 *   Query(flow)         -> pending batch handed over, then gns_{cm,ss}_query with n = 1
 *   Snapshot()          -> pending batch handed over, then cmHeavy's / the SS
 *                          HeavyHitters' sizing loop (capacity 64, grow, call again)
 *   Reset()             -> pending batch handed over, then gns_{cm,ss}_reset
 *
 * usage: gputask_replay <dir> ; <dir>/params.txt holds
 *   type width depth st_or_threshold ct m size base b nflow f0..f7 nelem e0..e7
 *   hll_master rng_seed batch_packets n_packets n_queries n_ops
 *   then n_ops lines "<packet index> <Q|R>"  (before packet i: Q = queries + snapshot, R = reset)
 * inputs  <dir>/{src16,dst16,sport,dport,proto,length,queries}.bin
 * output  <dir>/out.bin: for every Q (and once more at the end): the query answers
 *   (u64 each), then the heavy-hitter lists (CM: u64 nc, nc x (K flow bytes, u32),
 *   u64 ns, ns x (...); SS: u64 n, n x (...)); finally the exported state.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gns_sketch.h"

static void die(const char *what, int rc) {
    fprintf(stderr, "gputask_replay: %s failed (%d): %s\n", what, rc, gns_last_error());
    exit(2);
}
#define CK(call) do { int rc_ = (call); if (rc_ != GNS_OK) die(#call, rc_); } while (0)

static void *load(const char *dir, const char *name, size_t bytes) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "gputask_replay: cannot open %s\n", path); exit(2); }
    void *p = malloc(bytes ? bytes : 1);
    if (bytes && fread(p, 1, bytes, f) != bytes) { fprintf(stderr, "gputask_replay: short read %s\n", path); exit(2); }
    fclose(f);
    return p;
}

static uint32_t key_bytes(const gns_layout *l) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < l->n_fields; i++) {
        uint8_t f = l->fields[i];
        k += (f == GNS_F_SRCIP || f == GNS_F_DSTIP) ? 16 : (f == GNS_F_SRCPORT || f == GNS_F_DSTPORT) ? 2 : f == GNS_F_PROTO ? 1 : 0;
    }
    return k;
}

struct task {
    int type;
    gns_cm *cm;
    gns_ss *ss;
    uint32_t K;
    /* the pending host batch (GPUTask.cur) */
    uint8_t *src16, *dst16, *proto;
    uint16_t *sport, *dport;
    uint32_t *length;
    uint64_t fill, cap;
};

static void hand_over(struct task *t) {  /* GPUTask.handOverLocked + submitter.insert */
    if (t->fill == 0) return;
    gns_tuples tu = {t->src16, t->dst16, t->sport, t->dport, t->proto, t->length};
    if (t->type == 0) CK(gns_cm_insert_tuples(t->cm, &tu, t->fill, GNS_MEM_HOST));
    else CK(gns_ss_insert_tuples(t->ss, &tu, t->fill, GNS_MEM_HOST));
    t->fill = 0;
}

static void put_list(FILE *o, const uint8_t *flows, const uint32_t *v, uint64_t n, uint32_t K) {
    fwrite(&n, 8, 1, o);
    for (uint64_t i = 0; i < n; i++) {
        fwrite(flows + i * K, 1, K, o);
        fwrite(v + i, 4, 1, o);
    }
}

static void snapshot(struct task *t, FILE *o) {  /* cmHeavy / SuperSpread.HeavyHitters */
    uint64_t capC = 64, capS = 64;
    for (int tries = 0; tries < 8; tries++) {
        uint8_t *cf = malloc(capC * t->K + 1), *sf = malloc(capS * t->K + 1);
        uint32_t *cv = malloc(capC * 4 + 4), *sv = malloc(capS * 4 + 4);
        uint64_t nc = capC, ns = capS;
        if (t->type == 0) CK(gns_cm_heavy_hitters(t->cm, cf, cv, &nc, sf, sv, &ns));
        else CK(gns_ss_heavy_hitters(t->ss, cf, cv, &nc));
        if (nc > capC || (t->type == 0 && ns > capS)) {
            if (nc > capC) capC = 2 * nc;
            if (ns > capS) capS = 2 * ns;
            free(cf); free(sf); free(cv); free(sv);
            continue;
        }
        put_list(o, cf, cv, nc, t->K);
        if (t->type == 0) put_list(o, sf, sv, ns, t->K);
        free(cf); free(sf); free(cv); free(sv);
        return;
    }
    fprintf(stderr, "gputask_replay: heavy hitters did not settle\n");
    exit(2);
}

static void queries(struct task *t, const uint8_t *q, uint32_t nq, FILE *o) {  /* GPUTask.Query, one flow per call */
    for (uint32_t i = 0; i < nq; i++) {
        uint64_t v = 0;
        if (t->type == 0) CK(gns_cm_query(t->cm, q + (uint64_t)i * t->K, t->K, 1, &v));
        else CK(gns_ss_query(t->ss, q + (uint64_t)i * t->K, t->K, 1, &v));
        fwrite(&v, 8, 1, o);
    }
}

int main(int argc, char **argv) {
    if (argc != 2) { fprintf(stderr, "usage: %s <dir>\n", argv[0]); return 2; }
    const char *dir = argv[1];
    char path[4096];
    snprintf(path, sizeof path, "%s/params.txt", dir);
    FILE *pf = fopen(path, "r");
    if (!pf) { fprintf(stderr, "gputask_replay: no %s\n", path); return 2; }
    unsigned type, width, depth, thr, ct, m, size, nf, ne, f[8], e[8], batch, nq, nops;
    double base, b;
    unsigned long long hll, rng, n;
    if (fscanf(pf, "%u %u %u %u %u %u %u %lf %lf %u", &type, &width, &depth, &thr, &ct, &m, &size, &base, &b, &nf) != 10)
        return 2;
    for (int i = 0; i < 8; i++) if (fscanf(pf, "%u", &f[i]) != 1) return 2;
    if (fscanf(pf, "%u", &ne) != 1) return 2;
    for (int i = 0; i < 8; i++) if (fscanf(pf, "%u", &e[i]) != 1) return 2;
    if (fscanf(pf, "%llu %llu %u %llu %u %u", &hll, &rng, &batch, &n, &nq, &nops) != 6) return 2;
    uint64_t *op_at = calloc(nops + 1, 8);
    char *op = calloc(nops + 1, 1);
    for (unsigned i = 0; i < nops; i++) {
        char c[4];
        if (fscanf(pf, "%llu %3s", (unsigned long long *)&op_at[i], c) != 2) return 2;
        op[i] = c[0];
    }
    fclose(pf);

    struct task t;
    memset(&t, 0, sizeof t);
    t.type = (int)type;
    gns_layout fl = {nf, {0}}, el = {ne, {0}};
    for (int i = 0; i < 8; i++) { fl.fields[i] = (uint8_t)f[i]; el.fields[i] = (uint8_t)e[i]; }
    t.K = key_bytes(&fl);
    if (type == 0) {  /* NewCountMin(cfg.Width, cfg.Depth, cfg.SizeThreshold, cfg.CountThreshold, fields, K, nil, 0, Device) */
        gns_cm_params p;
        memset(&p, 0, sizeof p);
        p.width = width; p.depth = depth; p.size_threshold = thr; p.count_threshold = ct;
        p.flow = fl; p.key_bytes = t.K; p.seeds = NULL; p.max_flows = 0; p.device = 0;
        CK(gns_cm_create(&p, &t.cm));
    } else {  /* NewSuperSpread(W, D, CountThreshold, M, Size, Base, B, flow, elem, nil, hll, rng, 0, Device) */
        gns_ss_params p;
        memset(&p, 0, sizeof p);
        p.width = width; p.depth = depth; p.threshold = thr; p.m = m; p.size = size; p.base = base; p.b = b;
        p.flow = fl; p.elem = el; p.seeds = NULL; p.hll_master = hll; p.rng_seed = rng; p.max_flows = 0; p.device = 0;
        CK(gns_ss_create(&p, &t.ss));
    }
    const uint8_t *src16 = load(dir, "src16.bin", n * 16), *dst16 = load(dir, "dst16.bin", n * 16);
    const uint16_t *sport = load(dir, "sport.bin", n * 2), *dport = load(dir, "dport.bin", n * 2);
    const uint8_t *proto = load(dir, "proto.bin", n);
    const uint32_t *length = load(dir, "length.bin", n * 4);
    const uint8_t *q = load(dir, "queries.bin", (size_t)nq * t.K);
    t.cap = batch;
    t.src16 = malloc(16 * t.cap); t.dst16 = malloc(16 * t.cap);
    t.sport = malloc(2 * t.cap); t.dport = malloc(2 * t.cap); t.proto = malloc(t.cap); t.length = malloc(4 * t.cap);
    snprintf(path, sizeof path, "%s/out.bin", dir);
    FILE *o = fopen(path, "wb");
    if (!o) return 2;
    unsigned next = 0;
    for (uint64_t i = 0; i <= n; i++) {
        while (next < nops && op_at[next] == i) {
            hand_over(&t);
            if (op[next] == 'R') {
                if (type == 0) CK(gns_cm_reset(t.cm)); else CK(gns_ss_reset(t.ss));
            } else {
                queries(&t, q, nq, o);
                snapshot(&t, o);
            }
            next++;
        }
        if (i == n) break;
        /* ProcessPacket: append; a full batch is handed over */
        memcpy(t.src16 + 16 * t.fill, src16 + 16 * i, 16);
        memcpy(t.dst16 + 16 * t.fill, dst16 + 16 * i, 16);
        t.sport[t.fill] = sport[i]; t.dport[t.fill] = dport[i]; t.proto[t.fill] = proto[i]; t.length[t.fill] = length[i];
        if (++t.fill >= t.cap) hand_over(&t);
    }
    hand_over(&t);  /* Flush */
    queries(&t, q, nq, o);
    snapshot(&t, o);
    uint64_t cells = (uint64_t)(depth ? depth : 3) * (width ? width : (1u << 20));
    if (type == 0) {
        uint32_t *C = malloc(cells * 4), *S = malloc(cells * 4);
        uint8_t *Fc = malloc(cells * t.K), *Fs = malloc(cells * t.K);
        CK(gns_cm_flush(t.cm));
        CK(gns_cm_export_state(t.cm, C, S, Fc, Fs));
        fwrite(C, 4, cells, o); fwrite(S, 4, cells, o); fwrite(Fc, t.K, cells, o); fwrite(Fs, t.K, cells, o);
        CK(gns_cm_destroy(t.cm));
    } else {
        uint32_t mm = m ? m : 128;
        uint32_t *V = malloc(cells * 4);
        uint8_t *Kb = malloc(cells * t.K), *R = malloc(cells * mm);
        double *P = malloc(cells * 8);
        CK(gns_ss_flush(t.ss));
        CK(gns_ss_export_state(t.ss, V, Kb, R, P));
        fwrite(V, 4, cells, o); fwrite(Kb, t.K, cells, o); fwrite(R, 1, cells * mm, o); fwrite(P, 8, cells, o);
        CK(gns_ss_destroy(t.ss));
    }
    fclose(o);
    printf("gputask_replay: %llu packets, %u ops, ok\n", n, nops);
    return 0;
}
