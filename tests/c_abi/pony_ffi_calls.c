/*
 * pony_ffi_calls.c — calls every libgpuactor entry point the way a compiled
 * Pony program does (test infrastructure).
 *
 * The prototypes below are NOT taken from include/gpu_actor.h: they are the
 * C restatement of pony/gpu_actor/gpu_actor.pony's `use @...` declarations,
 * i.e. what gencall.c emits for a declared FFI call (gencall.c:1179-1198:
 * I32/U32/U64 -> i32/i32/i64 by value, Pointer[A]/struct/tag -> an opaque
 * pointer, a bare lambda -> a C function pointer). tests/test_c_abi_binary.py
 * checks them against both the Pony package and the header, and the struct
 * mirrors against the header's layout (pony_layout.c), so this binary linking
 * -lgpuactor and running is the ABI check a maintainer would otherwise only
 * get from ponyc.
 *
 *   pony_ffi_calls cpu          every entry point before init (no GPU needed)
 *   pony_ffi_calls gpu OUT.bin  message-ubench + spreader through the FFI,
 *                               states and counters written to OUT.bin for the
 *                               test to compare with the oracle
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pony_structs.h"

/* ---- gpu_actor.pony's declarations, as gencall.c lowers them ---- */
int32_t gpu_actor_init(void* cfg);
int32_t gpu_actor_shutdown(void);
int32_t gpu_actor_comm_id(void* out128);
int32_t gpu_actor_type_register(uint32_t type_id, uint32_t state_words, uint32_t table);
int32_t gpu_actor_type_config(uint32_t type_id, uint32_t batch, uint32_t mailbox_cap);
int32_t gpu_actor_type_priority(uint32_t type_id, int32_t priority);
int32_t gpu_actor_type_param(uint32_t type_id, uint32_t idx, uint64_t value);
int32_t gpu_actor_type_program(uint32_t type_id, void* code, uint32_t n);
int32_t gpu_actor_create(uint32_t type_id, uint64_t count, void* first);
int32_t gpu_actor_type_reserve(uint32_t type_id, uint64_t n);
int32_t gpu_actor_type_live(uint32_t type_id, void* live);
int32_t gpu_actor_alloc_msgs(uint64_t n, void* buf);
int32_t gpu_actor_sendv(void* first, uint64_t n);
int32_t gpu_actor_send(uint64_t to, uint32_t behaviour, uint64_t arg);
int32_t gpu_actor_run(uint64_t max_steps, void* steps_done);
int32_t gpu_actor_run_fixed(uint64_t n);
int32_t gpu_actor_run_async(uint64_t max_steps, void (*done)(void*, int32_t, uint64_t),
                            void* ctx);
int32_t gpu_actor_wait(void* steps_done);
int32_t gpu_actor_busy(void);
int32_t gpu_actor_sync(void);
int32_t gpu_actor_state_read(uint32_t type_id, uint64_t first, uint64_t n, void* out);
int32_t gpu_actor_state_write(uint32_t type_id, uint64_t first, uint64_t n, void* src);
int32_t gpu_actor_counts(void* out);
uint32_t gpu_actor_owner(uint64_t id);
const char* gpu_actor_strerror(int32_t code);
/* host-only entry points (not in the Pony package; C/ctypes callers) */
int32_t gpu_actor_set_transport(void* alltoallv, void* allreduce, void* ctx);
void* gpu_actor_stream(void);
double gpu_actor_last_drain_ms(void);

#define ESTATE (-6)
static int fails = 0;
#define EXPECT(expr, want) do { long long _v = (long long)(expr); \
  if(_v != (long long)(want)) { fprintf(stderr, "FAIL %s:%d %s = %lld, want %lld\n", \
    __FILE__, __LINE__, #expr, _v, (long long)(want)); ++fails; } } while(0)

static int cpu_mode(void)
{
  uint64_t u = 0, buf[8] = {0};
  pony_gpu_msg m[2] = {{0, 0, 1}, {1, 0, 2}};
  pony_gpu_msg* staging = NULL;
  pony_gpu_counts c;
  EXPECT(gpu_actor_shutdown(), ESTATE);
  EXPECT(gpu_actor_type_register(0, 3, 2), ESTATE);
  EXPECT(gpu_actor_type_config(0, 100, 16), ESTATE);
  EXPECT(gpu_actor_type_priority(0, 1), ESTATE);
  EXPECT(gpu_actor_type_param(0, 0, 1), ESTATE);
  EXPECT(gpu_actor_type_program(0, buf, 17), ESTATE);
  EXPECT(gpu_actor_create(0, 1, &u), ESTATE);
  EXPECT(gpu_actor_type_reserve(0, 1), ESTATE);
  EXPECT(gpu_actor_type_live(0, &u), ESTATE);
  EXPECT(gpu_actor_alloc_msgs(2, &staging), ESTATE);
  EXPECT(gpu_actor_sendv(m, 2), ESTATE);
  EXPECT(gpu_actor_send(0, 0, 0), ESTATE);
  EXPECT(gpu_actor_run(0, &u), ESTATE);
  EXPECT(gpu_actor_run_fixed(1), ESTATE);
  EXPECT(gpu_actor_run_async(0, NULL, NULL), ESTATE);
  EXPECT(gpu_actor_wait(&u), 0);
  EXPECT(gpu_actor_busy(), 0);
  EXPECT(gpu_actor_sync(), ESTATE);
  EXPECT(gpu_actor_state_read(0, 0, 1, buf), ESTATE);
  EXPECT(gpu_actor_state_write(0, 0, 1, buf), ESTATE);
  EXPECT(gpu_actor_counts(&c), ESTATE);
  EXPECT(gpu_actor_owner(7), 0);
  EXPECT(gpu_actor_set_transport(NULL, NULL, NULL), 0);        /* RCCL (default) */
  EXPECT(gpu_actor_stream() == NULL, 1);
  EXPECT(gpu_actor_last_drain_ms() == 0.0, 1);
  EXPECT(strcmp(gpu_actor_strerror(-9), "an asynchronous run is in flight"), 0);
  EXPECT(gpu_actor_init(NULL), -1);
  printf("cpu: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}

/* GpuRunDone's bare lambda (gpu_actor.pony): ctx is the notify actor */
static volatile int notified = 0;
static volatile int32_t notified_rc = -100;
static void run_done(void* ctx, int32_t rc, uint64_t steps)
{
  (void)steps;
  notified_rc = rc;
  *(volatile int*)ctx = 1;
}

#define N_PING 4096u
#define SPREAD_COUNT 10u

static int put(FILE* f, const void* p, size_t n)
{
  return fwrite(p, 1, n, f) == n ? 0 : 1;
}

static int gpu_mode(const char* out_path)
{
  pony_gpu_config cfg;
  memset(&cfg, 0, sizeof cfg);
  int32_t rc = gpu_actor_init(&cfg);
  if(rc != 0) { fprintf(stderr, "init: %s\n", gpu_actor_strerror(rc)); return 2; }
  uint8_t id[128];
  EXPECT(gpu_actor_comm_id(id), 0);

  /* message-ubench (examples/message-ubench/main.pony:223-286) */
  EXPECT(gpu_actor_type_register(0, 3, 2), 0);
  EXPECT(gpu_actor_type_config(0, 0, 16), 0);
  EXPECT(gpu_actor_type_priority(0, 0), 0);
  EXPECT(gpu_actor_type_param(0, 0, N_PING), 0);
  EXPECT(gpu_actor_type_param(0, 2, 20), 0);
  EXPECT(gpu_actor_type_param(0, 3, 5489), 0);
  uint64_t first = ~0ull;
  EXPECT(gpu_actor_create(0, N_PING, &first), 0);
  EXPECT(gpu_actor_type_param(0, 1, first), 0);
  pony_gpu_msg* chain = NULL;
  EXPECT(gpu_actor_alloc_msgs(5 * N_PING, &chain), 0);
  if(!chain) return 3;
  for(uint32_t k = 0; k < 5; ++k)
    for(uint32_t i = 0; i < N_PING; ++i)
    {
      chain[k * N_PING + i].to = (uint32_t)(first + i);
      chain[k * N_PING + i].behaviour = 0;
      chain[k * N_PING + i].arg = 42;
    }
  EXPECT(gpu_actor_sendv(chain, 5 * N_PING), 0);

  /* spreader (examples/spreader/main.pony:1-52) as a second type */
  EXPECT(gpu_actor_type_register(1, 5, 11), 0);
  EXPECT(gpu_actor_type_reserve(1, (1u << SPREAD_COUNT) - 2), 0);
  uint64_t root = ~0ull;
  EXPECT(gpu_actor_create(1, 1, &root), 0);
  EXPECT(gpu_actor_send(root, 0, (0xFFFFFFFFull << 32) | SPREAD_COUNT), 0);

  uint64_t steps = 0;
  EXPECT(gpu_actor_run(0, &steps), 0);
  uint64_t live = 0;
  EXPECT(gpu_actor_type_live(1, &live), 0);
  EXPECT(live, (1u << SPREAD_COUNT) - 1);
  pony_gpu_counts c1;
  EXPECT(gpu_actor_counts(&c1), 0);
  uint64_t* ps = calloc(3 * N_PING, 8);
  uint64_t* ss = calloc(5 * (size_t)live, 8);
  EXPECT(gpu_actor_state_read(0, 0, N_PING, ps), 0);
  EXPECT(gpu_actor_state_read(1, 0, live, ss), 0);

  /* second run: pony_sendi from the host, then run_async with the lambda */
  for(uint32_t j = 0; j < 3; ++j)
    EXPECT(gpu_actor_send(first + 7 * j, 0, 42), 0);
  volatile int flag = 0;
  EXPECT(gpu_actor_run_async(0, run_done, (void*)&flag), 0);
  uint64_t steps2 = 0;
  EXPECT(gpu_actor_wait(&steps2), 0);
  EXPECT(flag, 1);
  EXPECT(notified_rc, 0);
  EXPECT(gpu_actor_busy(), 0);
  pony_gpu_counts c2;
  EXPECT(gpu_actor_counts(&c2), 0);
  uint64_t* ps2 = calloc(3 * N_PING, 8);
  EXPECT(gpu_actor_state_read(0, 0, N_PING, ps2), 0);

  /* state_write round trip, fixed steps, the host-only helpers */
  EXPECT(gpu_actor_state_write(0, 0, N_PING, ps2), 0);
  EXPECT(gpu_actor_run_fixed(2), 0);
  EXPECT(gpu_actor_sync(), 0);
  EXPECT(gpu_actor_last_drain_ms() >= 0.0, 1);
  EXPECT(gpu_actor_stream() != NULL, 1);
  EXPECT(gpu_actor_owner(first + 3), 0);
  EXPECT(gpu_actor_set_transport(NULL, NULL, NULL), ESTATE);  /* only before init */

  FILE* f = fopen(out_path, "wb");
  int bad = !f;
  uint64_t hdr[4] = {steps, steps2, live, first};
  if(f)
  {
    bad |= put(f, hdr, sizeof hdr);
    bad |= put(f, &c1, sizeof c1);
    bad |= put(f, &c2, sizeof c2);
    bad |= put(f, ps, 3 * N_PING * 8);
    bad |= put(f, ss, 5 * live * 8);
    bad |= put(f, ps2, 3 * N_PING * 8);
    bad |= fclose(f) != 0;
  }
  free(ps); free(ss); free(ps2);
  EXPECT(gpu_actor_shutdown(), 0);
  EXPECT(gpu_actor_shutdown(), ESTATE);
  printf("gpu: %s (steps %llu + %llu)\n", (fails || bad) ? "FAILED" : "ok",
         (unsigned long long)steps, (unsigned long long)steps2);
  return (fails || bad) ? 1 : 0;
}

int main(int argc, char** argv)
{
  if(argc >= 2 && !strcmp(argv[1], "cpu")) return cpu_mode();
  if(argc >= 3 && !strcmp(argv[1], "gpu")) return gpu_mode(argv[2]);
  fprintf(stderr, "usage: %s cpu | gpu OUT.bin\n", argv[0]);
  return 64;
}
