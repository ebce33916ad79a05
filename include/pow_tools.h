/*
 * pow_tools.h — measurement helpers shipped with libpow_gpu.so (not part of
 * the reference's interface; used by bench.py for the roofline's peak).
 */
#ifndef POW_TOOLS_H
#define POW_TOOLS_H
#ifdef __cplusplus
extern "C" {
#endif

/* Instruction mixes of pow_valu_rate. */
enum {
  POW_VALU_MIX = 0,  /* K1's SHA-256 round stream (6 alignbit, 4 bitop3, 2 add3, 2 add: 8 half : 6 full rate) */
  POW_VALU_FULL = 1, /* v_bitop3_b32 + v_add_u32_e64, VGPR operands: full rate (the SIMD-32 ceiling) */
  POW_VALU_HALF = 2, /* v_alignbit_b32 + v_add3_u32: half rate */
};

typedef struct pow_valu_result {
  double lane_ops_per_s;   /* wave64 instructions x 64 / kernel time */
  double kernel_ms;        /* best of 3 timed runs (HIP events) */
  double clock_hz;         /* shader clock held during that run: s_memtime / s_memrealtime, median over workgroups */
  double cycles_per_instr; /* SIMD cycles per wave64 VALU instruction at that clock (2 = full rate on SIMD-32) */
} pow_valu_result;

/* Int32 VALU issue-rate microbenchmark on `device`: every CU runs 8 waves per
 * SIMD of 8 independent dependency chains per lane in the given mix.
 * Returns 0 or a POW_E* code. */
int pow_valu_rate(int device, int kind, pow_valu_result* res);
/* The same on a context's stream: the process holds no hardware queue more
 * (HIP keeps a stream's queue after the stream is destroyed, so
 * pow_valu_rate's own stream adds one for the process's lifetime). */
struct pow_ctx;
int pow_valu_rate_ctx(struct pow_ctx* ctx, int kind, pow_valu_result* res);

/* pow_valu_rate(device, POW_VALU_MIX): lane-ops/s and kernel time. */
int pow_valu_peak(int device, double* lane_ops_per_s, double* kernel_ms);

#ifdef __cplusplus
}
#endif
#endif
