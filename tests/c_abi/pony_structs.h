/* pony_structs.h — C mirrors of gpu_actor.pony's structs, field for field in
 * Pony declaration order (Pony lays a `struct` out as C does; ponyc
 * genprim/gentype). pony_layout.c checks them against include/gpu_actor.h. */
#ifndef PONY_STRUCTS_H
#define PONY_STRUCTS_H
#include <stdint.h>

typedef struct pony_gpu_msg        /* struct GpuMsg */
{
  uint32_t to;
  uint32_t behaviour;
  uint64_t arg;
} pony_gpu_msg;

typedef struct pony_gpu_config     /* struct GpuActorConfig */
{
  int32_t device;
  uint32_t n_ranks;
  uint32_t rank;
  uint32_t batch;
  uint32_t mailbox_cap;
  uint32_t max_exchange;
  uint64_t max_actors;
  void* comm_id;
} pony_gpu_config;

typedef struct pony_gpu_counts     /* struct GpuActorCounts (embed GpuTypeCounts) */
{
  uint64_t steps;
  uint64_t delivered;
  uint64_t sent;
  uint64_t pending;
  uint64_t dropped;
  uint64_t remote;
  uint64_t active;
  uint64_t delivered_by_type[16];
  uint64_t atomics;
} pony_gpu_counts;

#endif
