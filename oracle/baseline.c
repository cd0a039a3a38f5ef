/*
 * baseline.c — timed CPU verification of many (pub, msg, sig) triples, used only by
 * bench.py's cpu_baseline leg ("port" kind: this oracle's restatement of x/crypto's
 * ed25519.Verify, since the reference Go cannot be built here).
 * threads == 1 mirrors the single checkMaj23Routine goroutine (txflow/service.go:123-166).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 */
#include "oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <time.h>

typedef struct {
  const uint8_t *pubs, *arena, *sigs;
  const uint32_t *val_idx, *off;
  const uint16_t* len;
  uint8_t* out;
  uint32_t begin, end;
} job;

static void* run(void* p) {
  job* j = (job*)p;
  for (uint32_t i = j->begin; i < j->end; ++i)
    j->out[i] = (uint8_t)orc_ed25519_verify(j->pubs + 32 * (size_t)j->val_idx[i], j->arena + j->off[i],
                                            j->len[i], j->sigs + 64 * (size_t)i, 64);
  return 0;
}

static double now_s(void) {
  struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double orc_verify_many(const uint8_t* pubs32, const uint32_t* val_idx,
                       const uint8_t* msg_arena, const uint32_t* msg_off, const uint16_t* msg_len,
                       const uint8_t* sigs64, uint32_t n, int threads, uint8_t* out_ok) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  job jobs[256];
  pthread_t th[256];
  int started[256];
  double t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job){pubs32, msg_arena, sigs64, val_idx, msg_off, msg_len, out_ok,
                    (uint32_t)((uint64_t)n * t / threads), (uint32_t)((uint64_t)n * (t + 1) / threads)};
    started[t] = threads > 1 && pthread_create(&th[t], 0, run, &jobs[t]) == 0;   /* else inline */
    if (!started[t]) run(&jobs[t]);
  }
  for (int t = 0; t < threads; ++t)
    if (started[t]) pthread_join(th[t], 0);
  return now_s() - t0;
}
