// gns_ss.hip -- SuperSpread engine (super_spread.go).  Placeholder entry points
// until the device implementation lands; every call reports GNS_E_RANGE.
#include "gns_common.hpp"

using namespace gns;

#define SS_TODO() do { set_error("SuperSpread engine not built yet"); return GNS_E_RANGE; } while (0)

extern "C" {
int gns_ss_create(const gns_ss_params *, gns_ss **out) { if (out) *out = nullptr; SS_TODO(); }
int gns_ss_destroy(gns_ss *) { return GNS_OK; }
int gns_ss_insert_keys(gns_ss *, const uint8_t *, uint32_t, const uint8_t *, uint32_t, uint64_t, gns_mem) { SS_TODO(); }
int gns_ss_insert_tuples(gns_ss *, const gns_tuples *, uint64_t, gns_mem) { SS_TODO(); }
int gns_ss_insert_headers(gns_ss *, const uint8_t *, const uint32_t *, uint64_t, gns_mem) { SS_TODO(); }
int gns_ss_flush(gns_ss *) { SS_TODO(); }
int gns_ss_query(gns_ss *, const uint8_t *, uint32_t, uint64_t, uint64_t *) { SS_TODO(); }
int gns_ss_heavy_hitters(gns_ss *, uint8_t *, uint32_t *, uint64_t *) { SS_TODO(); }
int gns_ss_reset(gns_ss *) { SS_TODO(); }
int gns_ss_export_state(gns_ss *, uint32_t *, uint8_t *, uint8_t *, double *) { SS_TODO(); }
int gns_ss_stats(gns_ss *, uint64_t *) { SS_TODO(); }
int gns_ss_set_timing(gns_ss *, int) { SS_TODO(); }
int gns_ss_stage_times(gns_ss *, double *, uint64_t *, int) { SS_TODO(); }
}
