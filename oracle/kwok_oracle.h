/* kwok_oracle.h - CPU oracle (TEST INFRASTRUCTURE ONLY; see kwok_oracle.c).
 * Same record layout and call sequence as the product's C-ABI
 * (include/kwok_engine.h), so one harness drives both. */
#ifndef KWOK_ORACLE_H
#define KWOK_ORACLE_H
#include "../include/kwok_engine.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct kwok_oracle kwok_oracle;
int kwok_oracle_create(const kwok_config* cfg, kwok_oracle** out);
void kwok_oracle_destroy(kwok_oracle* o);
const char* kwok_oracle_last_error(const kwok_oracle* o);
int kwok_oracle_register_pod_spec(kwok_oracle* o, const kwok_pod_spec* spec, const char* arena, size_t arena_len,
                                  int32_t* out_id);
int kwok_oracle_ingest_nodes(kwok_oracle* o, const kwok_node_event* ev, size_t n, const char* arena, size_t arena_len,
                             int32_t* out_handles, int32_t* out_status);
int kwok_oracle_ingest_pods(kwok_oracle* o, const kwok_pod_event* ev, size_t n, const char* arena, size_t arena_len,
                            int32_t* out_handles, int32_t* out_status, uint32_t* out_released);
int kwok_oracle_ingest_pods_packed(kwok_oracle* o, const kwok_pod_rec* recs, size_t n, int32_t* out_handles,
                                   int8_t* out_status, uint32_t* out_released);
int kwok_oracle_ingest_pods_packed12(kwok_oracle* o, const kwok_pod_rec12* recs, size_t n, int32_t* out_new_handles,
                                     size_t new_cap, int8_t* out_status, uint32_t* out_released);
int kwok_oracle_pool_put(kwok_oracle* o, const uint32_t* ips, size_t n);
int kwok_oracle_cni_pending(kwok_oracle* o, int32_t* out, size_t cap, size_t* n_out);
int kwok_oracle_cni_assign(kwok_oracle* o, const int32_t* handles, const uint32_t* ips, size_t n, int32_t* out_status);
int kwok_oracle_tick(kwok_oracle* o, int64_t now_unix, kwok_tick_result* res);
/* host threads of the tick's per-object sweeps (<= 0: all; 1: sequential); returns the count */
int kwok_oracle_set_threads(kwok_oracle* o, int n);
int kwok_oracle_read_outputs(kwok_oracle* o, kwok_outputs* out);
int kwok_oracle_read_arena(kwok_oracle* o, uint64_t off, uint64_t len, void* dst);
int kwok_oracle_node_has(kwok_oracle* o, const char* name, size_t len);
uint64_t kwok_oracle_node_size(kwok_oracle* o);
int kwok_oracle_dump_pods(kwok_oracle* o, int32_t first, uint32_t count, uint8_t* used, uint8_t* phase,
                          uint32_t* host_ip, uint32_t* pod_ip);
#ifdef __cplusplus
}
#endif
#endif
