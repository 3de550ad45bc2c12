// Lab (not product code): aggregate host memcpy bandwidth with T threads, each copying its own
// 256 MiB buffers R times (first-touch by the copying thread). Usage: memcpy_bw T R
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static size_t N = 256u << 20;
static int R = 4;
static pthread_barrier_t bar;
static volatile unsigned long long sink;
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }
static void *run(void *arg) {
  (void)arg;
  char *a = malloc(N), *b = malloc(N);
  memset(a, 1, N); memset(b, 2, N);
  pthread_barrier_wait(&bar);
  for (int r = 0; r < R; r++) { memcpy(b, a, N); sink += (unsigned char)b[r * 4096 % N]; a[r] ^= 1; }
  pthread_barrier_wait(&bar);
  free(a); free(b);
  return NULL;
}
int main(int argc, char **argv) {
  int T = argc > 1 ? atoi(argv[1]) : 16;
  R = argc > 2 ? atoi(argv[2]) : 4;
  pthread_t th[256];
  pthread_barrier_init(&bar, NULL, T + 1);
  for (int i = 0; i < T; i++) pthread_create(&th[i], NULL, run, NULL);
  pthread_barrier_wait(&bar);
  double t0 = now();
  pthread_barrier_wait(&bar);
  double t = now() - t0;
  for (int i = 0; i < T; i++) pthread_join(th[i], NULL);
  printf("threads %d: %.1f GB/s copied (%.2f GB in %.3f s)\n", T, (double)T * R * N / t / 1e9, (double)T * R * N / 1e9, t);
  return 0;
}
