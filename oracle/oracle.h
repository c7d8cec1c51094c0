/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of (1) the workload RNGs the BASELINE workloads draw from and
 * (2) a single-threaded bulk-synchronous (BSP) simulator of the gpu_actor engine
 * semantics. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load liboracle.so, and only as the checker: the product
 * (ponyc_amd/libgpuactor.so) never links or calls anything here.
 *
 * Parity is pinned two ways (see DESIGN.md "Oracle"):
 *   - RNGs against the reference's own KATs (packages/random/_test.pony);
 *   - BSP final states against golden fixtures produced by the reference
 *     runtime itself (oracle/_ref/libponyrt.so + oracle/harness/ drivers).
 */
#ifndef ORACLE_H
#define ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG restatements ------------------------------------------------- */

/* 64x64 -> high 64 bits; Random.int() on native128 (random.pony:143-156). */
uint64_t or_mulhi(uint64_t a, uint64_t b);

/* XorOshiro128Plus (packages/random/xoroshiro.pony:1-42). create(x, y) stores
 * the state and calls next() once (xoroshiro.pony:22-29). */
typedef struct { uint64_t x, y; } or_xoro_t;
void     or_xoro_create(or_xoro_t* r, uint64_t x, uint64_t y);
uint64_t or_xoro_next(or_xoro_t* r);
uint64_t or_rand_int(or_xoro_t* r, uint64_t n);            /* random.pony:143-156 */
uint64_t or_rand_int_unbiased(or_xoro_t* r, uint64_t n);   /* random.pony:159-193 */

/* SplitMix64 (packages/random/splitmix64.pony). */
uint64_t or_splitmix_next(uint64_t* state);
/* Stateless form: next() of a SplitMix64 freshly seeded with x. */
uint64_t or_splitmix_mix(uint64_t x);

/* PolyRand (examples/gups_basic/main.pony:167-216). */
typedef struct { uint64_t last; } or_polyrand_t;
void     or_polyrand_create(or_polyrand_t* r, uint64_t seed);
uint64_t or_polyrand_next(or_polyrand_t* r);
uint64_t or_gups_update_xor(uint64_t streamers, uint64_t chunk, uint64_t iterate);
uint64_t or_gups_update_xor_literal(uint64_t streamers, uint64_t chunk, uint64_t iterate);

/* ---- BSP simulator ------------------------------------------------------ */
/* Mirrors include/gpu_actor.h (same handler tables, behaviour ids, state
 * layouts and type params), restated independently in C. Semantics: step s
 * runs actors in ascending id order; each processes min(batch, pending-at-
 * step-start) messages from the head of its mailbox; an emitted message is
 * appended to the receiver's mailbox (visible from step s+1). Messages to a
 * type whose behaviours are all commutative ("reducible") are applied when
 * sent. Host sends are appended after all actor emissions of the window. */
int  or_init(uint32_t n_types_max);
void or_shutdown(void);
int  or_type_register(uint32_t type_id, uint32_t state_words, uint32_t ht);
int  or_type_config(uint32_t type_id, uint32_t batch, uint32_t mailbox_cap);
int  or_type_priority(uint32_t type_id, int32_t priority);
int  or_type_param(uint32_t type_id, uint32_t idx, uint64_t value);
int  or_type_program(uint32_t type_id, const uint64_t* code, uint32_t n);
int  or_create(uint32_t type_id, uint64_t count, uint64_t* first_id);
/* room for n actors created by behaviours (before or_create); live count */
int  or_type_reserve(uint32_t type_id, uint64_t n);
int  or_type_live(uint32_t type_id, uint64_t* out);
int  or_send(uint64_t to, uint32_t behaviour, uint64_t arg);
int  or_sendv(const void* msgs, uint64_t n);   /* msgs: gpu_msg_t[n] */
int  or_run(uint64_t max_steps, uint64_t* steps_done);
int  or_state_read(uint32_t type_id, uint64_t first, uint64_t n, uint64_t* out);
int  or_state_write(uint32_t type_id, uint64_t first, uint64_t n, const uint64_t* in);
/* counts: [0]=steps [1]=delivered [2]=sent [3]=pending [4]=dropped */
uint64_t or_trig_count(void);
int  or_counts(uint64_t* out5);
int  or_type_delivered(uint32_t type_id, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
