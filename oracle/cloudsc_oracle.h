/*
 * cloudsc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference CLOUDSC kernel
 * (src/cloudsc_c/cloudsc/cloudsc_c.c:19-2587 of lukasm91/dwarf-p-cloudsc).
 * It is the checker for the HIP kernels and the "port" CPU baseline of
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it; the product library (libcloudsc_amd.so) never links it.
 *
 * Parity pinning: tests/test_oracle.py checks it bit-for-bit against the
 * reference C kernel compiled from /root/reference (oracle/_ref, recipe in
 * oracle/Makefile) and against the reference goldens (tests/golden/, copied
 * from data/reference_*.dat == config-files/reference.h5).
 */
#ifndef CLOUDSC_ORACLE_H
#define CLOUDSC_ORACLE_H
#include "cloudsc_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One NPROMA block (block-local pointers, klon = nproma), columns kidia..kfdia
 * (1-based, inclusive, as cloudsc_c()).  Writes every output element of the
 * processed columns (see cloudsc_amd.h output contract). */
int cloudsc_oracle_block_dp(const cloudsc_params_t *p, int kidia, int kfdia, int klon, int klev,
                            const cloudsc_fields_t *f);
int cloudsc_oracle_block_sp(const cloudsc_params_t *p, int kidia, int kfdia, int klon, int klev,
                            const cloudsc_fields_t *f);

/* Whole problem in block layout, OpenMP over blocks with schedule(runtime)
 * (cloudsc_driver.c:183-217).  precision = CLOUDSC_FP64 or CLOUDSC_FP32.
 * Returns wall seconds of the block loop in *seconds (may be NULL). */
int cloudsc_oracle_run(int nthreads, int precision, int ngptot, int nproma, int klev,
                       const cloudsc_params_t *p, const cloudsc_fields_t *f, double *seconds);

/* Sensitivity probe of the fp32 restatement: seed != 0 moves every expf/powf
 * result by -1, 0 or +1 ulp (a hash of the arguments and the seed picks which);
 * 0 restores the plain C library results.  Not thread-safe against a running
 * cloudsc_oracle_run. */
void cloudsc_oracle_set_libm_nudge(unsigned seed);

#ifdef __cplusplus
}
#endif
#endif
