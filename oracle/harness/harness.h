/*
 * harness.h — TEST INFRASTRUCTURE ONLY. Shared scaffolding for the C drivers
 * that rebuild the BASELINE workloads' actor graphs on the reference runtime's
 * public ABI (pony.h), the way ponyc-generated code calls it:
 *   - an actor type is a pony_type_t {id, size, ..., dispatch}
 *     (pony.h:171-195) whose instances are pony_actor_pad_t + fields
 *     (pony.h:232-250);
 *   - a behaviour call is pony_alloc_msg + pony_sendv (gencall.c:524-626),
 *     here via the pony_sendi/pony_sendp conveniences (actor.c:941-968);
 *   - main() = pony_init; pony_become(holder); create + send; pony_start
 *     (genexe.c:97-230).
 * Actors are created while a holder actor is "become"d so they start with
 * rc = GC_INC_MORE (actor.c:719-727) and survive --ponynoblock reaping.
 * Final per-actor state: the runtime owns actor memory after pony_start. An
 * actor it destroys runs its type's finaliser first (ponyint_actor_final,
 * actor.c:628-640), which copies the state out and marks the actor's slot
 * (h_fin); every unmarked actor is still live and is read in place. Nothing
 * is copied per behaviour, so timed runs do only the reference's work.
 */
#ifndef HARNESS_H
#define HARNESS_H

#define _GNU_SOURCE
#include <pony.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <time.h>

#include "oracle.h"

/* runtime_options override the generated program would provide (start.c:99) */
struct options_t;
void Main_runtime_override_defaults_oo(struct options_t* opt) { (void)opt; }

static inline double h_now(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

/* --key value argument lookup (ints only) */
static inline uint64_t h_arg(int argc, char** argv, const char* key, uint64_t dflt)
{
  for(int i = 1; i + 1 < argc; i++)
    if(strcmp(argv[i], key) == 0)
      return strtoull(argv[i + 1], NULL, 0);
  return dflt;
}

static inline const char* h_sarg(int argc, char** argv, const char* key, const char* dflt)
{
  for(int i = 1; i + 1 < argc; i++)
    if(strcmp(argv[i], key) == 0)
      return argv[i + 1];
  return dflt;
}

/* Holder actor: never receives anything, only "become"d on the main thread. */
typedef struct { pony_actor_pad_t pad; } holder_t;
static void holder_dispatch(pony_ctx_t* ctx, pony_actor_t* self, pony_msg_t* m)
{ (void)ctx; (void)self; (void)m; }
static pony_type_t holder_type = { .id = 0, .size = sizeof(holder_t),
  .dispatch = holder_dispatch };

/* Start the runtime with --ponymaxthreads=T --ponynoblock (+ --ponynoscale
 * when asked) and become the holder actor. Returns the context. */
static inline pony_ctx_t* h_start(int threads, int noscale)
{
  static char a0[] = "harness", a1[64], a2[] = "--ponynoblock", a3[] = "--ponynoscale";
  snprintf(a1, sizeof(a1), "--ponymaxthreads=%d", threads);
  char* av[] = { a0, a1, a2, a3, NULL };
  int ac = noscale ? 4 : 3;
  pony_init(ac, av);
  pony_ctx_t* ctx = pony_ctx();
  pony_actor_t* holder = pony_create(ctx, &holder_type);
  pony_become(ctx, holder);
  return ctx;
}

/* Run to quiescence; returns seconds spent in pony_start. */
static inline double h_run(pony_ctx_t* ctx)
{
  pony_become(ctx, NULL);
  double t0 = h_now();
  int ec = 0;
  pony_start(false, &ec, NULL);
  return h_now() - t0;
}

/* Slots whose actor the runtime finalised (its state already copied out). */
static unsigned char* h_fin;

/* Write `words` field-major arrays of n u64 to path (raw little-endian). */
static inline int h_dump(const char* path, const uint64_t* const* fields, int words, uint64_t n)
{
  if(path == NULL || path[0] == 0) return 0;
  FILE* f = fopen(path, "wb");
  if(!f) { perror(path); return 1; }
  for(int w = 0; w < words; w++)
    fwrite(fields[w], sizeof(uint64_t), n, f);
  fclose(f);
  return 0;
}

/* One JSON line of timing on stdout, consumed by bench.py / gen scripts. */
static inline void h_report(const char* name, int threads, double secs, uint64_t msgs)
{
  printf("{\"harness\": \"%s\", \"threads\": %d, \"seconds\": %.6f, \"msgs\": %llu, "
    "\"msgs_per_sec\": %.1f}\n", name, threads, secs, (unsigned long long)msgs,
    secs > 0 ? (double)msgs / secs : 0.0);
  fflush(stdout);
}

#endif
