#include <stdio.h>
#include <time.h>
#include "pow_gpu.h"
static double now(){struct timespec t; clock_gettime(CLOCK_MONOTONIC,&t); return t.tv_sec+1e-9*t.tv_nsec;}
int main(){
  double t0=now(); int n=0; pow_device_count(&n); double t1=now();
  pow_ctx* a; pow_init(0,&a); double t2=now();
  pow_ctx* b; pow_init(0,&b); double t3=now();
  pow_warmup(a); double t4=now(); pow_warmup(b); double t5=now();
  printf("{\"device_count_ms\": %.1f, \"init1_ms\": %.1f, \"init2_ms\": %.1f, \"warmup1_ms\": %.1f, \"warmup2_ms\": %.1f}\n",
    1e3*(t1-t0),1e3*(t2-t1),1e3*(t3-t2),1e3*(t4-t3),1e3*(t5-t4));
  return 0;
}
