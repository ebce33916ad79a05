/*
 * pow_tools.h — measurement helpers shipped with libpow_gpu.so (not part of
 * the reference's interface; used by bench.py for the roofline's peak).
 */
#ifndef POW_TOOLS_H
#define POW_TOOLS_H
#ifdef __cplusplus
extern "C" {
#endif

/* Int32 VALU throughput microbenchmark on `device`: every CU runs 8 waves per
 * SIMD of independent v_alignbit_b32 / v_bitop3_b32 / v_add3_u32 chains (the
 * SHA-256 instruction mix).  Outputs lane-ops/s (one wave64 instruction = 64
 * lane-ops) and the kernel time.  Returns 0 or a POW_E* code. */
int pow_valu_peak(int device, double* lane_ops_per_s, double* kernel_ms);

#ifdef __cplusplus
}
#endif
#endif
