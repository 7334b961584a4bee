/* One mchecksum object, reset/update(n bytes)/get repeated: GB/s of the CPU
 * streaming path for one method and update size (tools/cpu_paths.sh). */
#include <mchecksum.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <time.h>
static double now(void){struct timespec t; clock_gettime(CLOCK_MONOTONIC,&t); return t.tv_sec+t.tv_nsec*1e-9;}
int main(int argc, char **argv){
  const char *m = argv[1]; size_t n = strtoull(argv[2],0,10); int reps = atoi(argv[3]);
  uint8_t *b = malloc(n+64); for (size_t i=0;i<n+64;i++) b[i]=(uint8_t)(i*131+7);
  mchecksum_object_t c; mchecksum_init(m,&c); uint64_t h=0;
  double t0=now();
  for (int r=0;r<reps;r++){ mchecksum_reset(c); mchecksum_update(c,b,n); mchecksum_get(c,&h,8,1);}
  double el=now()-t0; printf("%s n=%zu %.2f GB/s\n", m, n, (double)n*reps/el/1e9);
  return 0; }
