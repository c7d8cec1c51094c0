/* pony_layout.c — compile-time check that gpu_actor.pony's structs (mirrored
 * in pony_structs.h) have the header's size and field offsets. Compiled,
 * never run: a mismatch is a build error. */
#include <stddef.h>
#include "gpu_actor.h"
#include "pony_structs.h"

#define SAME(P, H, f) _Static_assert(offsetof(P, f) == offsetof(H, f), #P "." #f)

_Static_assert(sizeof(pony_gpu_msg) == sizeof(gpu_msg_t), "GpuMsg size");
SAME(pony_gpu_msg, gpu_msg_t, to);
SAME(pony_gpu_msg, gpu_msg_t, behaviour);
SAME(pony_gpu_msg, gpu_msg_t, arg);
_Static_assert(sizeof(pony_gpu_msg) == 2 * sizeof(uint64_t), "GpuMsgs packs 2 x U64");

_Static_assert(sizeof(pony_gpu_config) == sizeof(gpu_actor_config_t), "config size");
SAME(pony_gpu_config, gpu_actor_config_t, device);
SAME(pony_gpu_config, gpu_actor_config_t, n_ranks);
SAME(pony_gpu_config, gpu_actor_config_t, rank);
SAME(pony_gpu_config, gpu_actor_config_t, batch);
SAME(pony_gpu_config, gpu_actor_config_t, mailbox_cap);
SAME(pony_gpu_config, gpu_actor_config_t, max_exchange);
SAME(pony_gpu_config, gpu_actor_config_t, max_actors);
SAME(pony_gpu_config, gpu_actor_config_t, comm_id);

_Static_assert(sizeof(pony_gpu_counts) == sizeof(gpu_actor_counts_t), "counts size");
SAME(pony_gpu_counts, gpu_actor_counts_t, steps);
SAME(pony_gpu_counts, gpu_actor_counts_t, delivered);
SAME(pony_gpu_counts, gpu_actor_counts_t, sent);
SAME(pony_gpu_counts, gpu_actor_counts_t, pending);
SAME(pony_gpu_counts, gpu_actor_counts_t, dropped);
SAME(pony_gpu_counts, gpu_actor_counts_t, remote);
SAME(pony_gpu_counts, gpu_actor_counts_t, active);
SAME(pony_gpu_counts, gpu_actor_counts_t, delivered_by_type);
SAME(pony_gpu_counts, gpu_actor_counts_t, atomics);

int pony_layout_checked(void) { return 1; }
