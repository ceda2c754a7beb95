/*
 * cloudsc_amd.h -- C ABI of the MI355X-native CLOUDSC dwarf (libcloudsc_amd.so).
 *
 * Plain C: no C++ or torch types, plain pointers and sizes.  Every entry point
 * returns 0 on success or a negative CLOUDSC_E* code; the library never calls
 * exit().  Parameters live in per-parameter-set device blocks: each device has
 * a default set (cloudsc_gpu_init, used by cloudsc_gpu_run), and every state
 * and host pipeline owns a private copy, so states with different parameters
 * can be interleaved on one device.  One host thread per device -- or one
 * thread driving N devices -- is safe.  cloudsc_gpu_init rewrites the device's
 * default set in place: it must not race with cloudsc_gpu_run or
 * cloudsc_host_pipeline_create on the same device from another thread (states
 * and pipelines already created are unaffected).
 *
 * Which reference interface each declaration replaces (paths relative to the
 * lukasm91/dwarf-p-cloudsc checkout):
 *
 *   cloudsc_params_t   <- struct TECLDP (src/cloudsc_c/cloudsc/yoecldp_c.h:21-141)
 *                         + YOMCST globals (yomcst_c.h:14-72) + YOETHF globals
 *                         (yoethf_c.h:14-36) + PTSPHY, filled by load_state()
 *                         (src/cloudsc_c/cloudsc/load_state.c:538-690)
 *   cloudsc_fields_t   <- the 56 array arguments of cloudsc_c()
 *                         (src/cloudsc_c/cloudsc/cloudsc_c.h:18-29) and of the
 *                         CUDA kernel (src/cloudsc_cuda/cloudsc/cloudsc_c_k_caching.cu:13-40)
 *   cloudsc_gpu_init   <- cudaMemcpy of the TECLDP struct + the 28 by-value
 *                         constants (src/cloudsc_cuda/cloudsc/cloudsc_driver.cu:312,383,412-416)
 *   cloudsc_gpu_check  <- the cudaPeekAtLastError/cudaDeviceSynchronize check
 *                         after the launch (cloudsc_driver.cu:419-420)
 *   cloudsc_cpu_run    <- the CPU dwarf's OpenMP block loop calling cloudsc_c()
 *                         (src/cloudsc_c/cloudsc/cloudsc_driver.c:183-217, kernel
 *                         cloudsc_c.c:19-2587, declared cloudsc_c.h:18-29)
 *   cloudsc_gpu_run    <- cloudsc_c<<<grid,nproma>>>(...) (cloudsc_driver.cu:391-416)
 *   cloudsc_state_*    <- the driver plumbing around the kernel: load+expand
 *                         (load_state.c:69-184,279), timing (cloudsc_driver.c:181-262),
 *                         validation (src/common/module/validate_mod.F90:118-296)
 *
 * Field layout (identical to the reference C/CUDA drivers, cloudsc_driver.c:114-171):
 * NPROMA-blocked, nblocks = ceil(ngptot/nproma), column jl of block b is global
 * column b*nproma+jl.
 *   full-level field     [nblocks][klev][nproma]
 *   half-level field     [nblocks][klev+1][nproma]      (paph, the 14 flux fields)
 *   species field        [nblocks][NCLV][klev][nproma]  (pclv, tendency_*_cld)
 *   surface field        [nblocks][nproma]              (plsm, ktype, prainfrac_toprfz)
 * Element type is double for CLOUDSC_FP64 and float for CLOUDSC_FP32 (ktype is
 * always int32).  Lanes jl >= bsize of the last block are never read or written.
 *
 * Output contract (stronger than the reference C kernel, matches the CUDA one):
 * the callee writes EVERY output element of every active column -- including
 * tendency_loc_cld[vapour] (zero) and pcovptot at levels < NCLDTOP (zero) --
 * so the caller need not pre-zero (cf. cloudsc_driver.c:199-200).  plude is
 * read-modify-write exactly as in the reference (cloudsc_c.c:970,980).
 */
#ifndef CLOUDSC_AMD_H
#define CLOUDSC_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define CLOUDSC_NCLV 5          /* ql, qi, qr, qs, qv (yoecldp_c.h:13-18)            */

/* precision selector */
#define CLOUDSC_FP64 8
#define CLOUDSC_FP32 4

/* kernel variant selector */
#define CLOUDSC_VARIANT_SCC    1   /* SCC baseline: level phases as separate sweeps, temporaries in HBM scratch */
#define CLOUDSC_VARIANT_KCACHE 2   /* SCC-k-caching: one fused level loop, carried state in registers       */
#define CLOUDSC_VARIANT_KSEG   3   /* SCC-k-caching, persistent work queue over (level segment, block)      */
                                   /* items; carried state handed between segments through HBM scratch   */
#define CLOUDSC_VARIANT_SCC_PRIVATE 4  /* SCC with per-thread private-array temporaries (scratch memory):   */
                                   /* the reference CUDA SCC form, cloudsc_c.cu:60-317; klev <= 137 as    */
                                   /* there (:53); no caller workspace                                     */

/* Option bit, OR-ed into a `variant` argument (cloudsc_gpu_run, cloudsc_state_run,
 * cloudsc_host_pipeline_run).  fp32 evaluates exp/pow in single precision with
 * the device's float forms by default (hardware exp2/log2 with an exact
 * argument reduction: <= 2 ulp, every operation float) and divides with the
 * hardware reciprocal and one residual correction (within 1 ulp); with this
 * bit it uses the reference CPU build's glibc expf/powf algorithms (computed in
 * double) and correctly rounded divisions instead: bit-identical to the
 * single-precision restatement, slower.  fp64 always uses the reference CPU
 * build's exp/pow and IEEE divisions and ignores the bit. */
#define CLOUDSC_FP32_EXACT_LIBM 0x100

/* error codes */
#define CLOUDSC_OK            0
#define CLOUDSC_EINVAL      (-1)   /* bad argument (sizes, NULL pointer, precision, variant) */
#define CLOUDSC_ENODEV      (-2)   /* no such HIP device                                      */
#define CLOUDSC_EHIP        (-3)   /* a HIP runtime call failed (see cloudsc_last_hip_error) */
#define CLOUDSC_ENOINIT     (-4)   /* cloudsc_gpu_init not called for this device           */
#define CLOUDSC_ENOMEM      (-5)   /* device or host allocation failed                        */
#define CLOUDSC_EIO         (-6)   /* file could not be read / wrong format                   */
#define CLOUDSC_EHANDOFF    (-7)   /* a KSEG segment hand-off timed out: outputs invalid      */

/* ------------------------------------------------------------------------ */
/* Parameters: YOMCST + YOETHF + TECLDP (without rbeta/rbetap1) + PTSPHY     */
/* ------------------------------------------------------------------------ */
typedef struct cloudsc_params {
  double ptsphy;
  /* YOMCST (the 9 the kernel reads) */
  double rg, rd, rcpd, retv, rlvtt, rlstt, rlmlt, rtt, rv;
  /* YOETHF */
  double r2es, r3les, r3ies, r4les, r4ies, r5les, r5ies, r5alvcp, r5alscp;
  double ralvdcp, ralsdcp, ralfdcp, rtwat, rtice, rticecu, rtwat_rtice_r, rtwat_rticecu_r;
  double rkoop1, rkoop2;
  /* TECLDP doubles, in yoecldp_c.h order */
  double ramid, rcldiff, rcldiff_convi, rclcrit, rclcrit_sea, rclcrit_land, rkconv, rprc1, rprc2;
  double rcldmax, rpecons, rvrfactor, rprecrhmax, rtaumel, ramin, rlmin, rkooptau, rcldtopp;
  double rlcritsnow, rsnowlin1, rsnowlin2, ricehi1, ricehi2, riceinit, rvice, rvrain, rvsnow;
  double rthomo, rcovpmin, rccn, rnice, rccnom, rccnss, rccnsu, rcldtopcf, rdepliqrefrate;
  double rdepliqrefdepth, rcl_kkaac, rcl_kkbac, rcl_kkaau, rcl_kkbauq, rcl_kkbaun;
  double rcl_kk_cloud_num_sea, rcl_kk_cloud_num_land, rcl_ai, rcl_bi, rcl_ci, rcl_di;
  double rcl_x1i, rcl_x2i, rcl_x3i, rcl_x4i, rcl_const1i, rcl_const2i, rcl_const3i, rcl_const4i;
  double rcl_const5i, rcl_const6i, rcl_apb1, rcl_apb2, rcl_apb3, rcl_as, rcl_bs, rcl_cs, rcl_ds;
  double rcl_x1s, rcl_x2s, rcl_x3s, rcl_x4s, rcl_const1s, rcl_const2s, rcl_const3s, rcl_const4s;
  double rcl_const5s, rcl_const6s, rcl_const7s, rcl_const8s, rdenswat, rdensref, rcl_ar, rcl_br;
  double rcl_cr, rcl_dr, rcl_x1r, rcl_x2r, rcl_x4r, rcl_ka273, rcl_cdenom1, rcl_cdenom2, rcl_cdenom3;
  double rcl_schmidt, rcl_dynvisc, rcl_const1r, rcl_const2r, rcl_const3r, rcl_const4r, rcl_fac1;
  double rcl_fac2, rcl_const5r, rcl_const6r, rcl_fzrab, rcl_fzrbb, nshapep, nshapeq;
  /* TECLDP integers / logicals (logical: 0 = .FALSE., nonzero = .TRUE.) */
  int lcldextra, lcldbudget, nssopt, ncldtop;
  int naeclbc, naecldu, naeclom, naeclss, naeclsu, nclddiag, naercld;
  int laerliqautolsp, laerliqautocp, laerliqautocpb, laerliqcoll, laericesed, laericeauto;
  int nbeta;
} cloudsc_params_t;

/* ------------------------------------------------------------------------ */
/* Field pointers (device pointers for cloudsc_gpu_run)                      */
/* ------------------------------------------------------------------------ */
typedef struct cloudsc_fields {
  /* inputs */
  const void *pt, *pq;
  const void *tendency_tmp_t, *tendency_tmp_q, *tendency_tmp_a, *tendency_tmp_cld;
  const void *pvfl, *pvfi, *phrsw, *phrlw, *pvervel, *pap, *paph, *plsm;
  const int  *ktype;
  const void *plu, *psnde, *pmfu, *pmfd, *pa, *pclv, *psupsat;
  /* aerosol inputs: read only when the matching LAER* flag is set; may be NULL otherwise */
  const void *plcrit_aer, *picrit_aer, *pre_ice, *pccn, *pnice;
  /* in/out */
  void *plude;
  /* outputs */
  void *tendency_loc_t, *tendency_loc_q, *tendency_loc_a, *tendency_loc_cld;
  void *pcovptot, *prainfrac_toprfz;
  void *pfsqlf, *pfsqif, *pfcqnng, *pfcqlng, *pfsqrf, *pfsqsf, *pfcqrng, *pfcqsng;
  void *pfsqltur, *pfsqitur, *pfplsl, *pfplsn, *pfhpsl, *pfhpsn;
} cloudsc_fields_t;

/* ------------------------------------------------------------------------ */
/* Low-level boundary: run the kernel on caller-owned device buffers         */
/* ------------------------------------------------------------------------ */

/* Number of visible HIP devices. */
int cloudsc_gpu_device_count(int *count);

/* Set the device's default parameter set (fp64 and fp32 mirrors, folded on
 * the host) used by cloudsc_gpu_run.  Must be called once per device before
 * cloudsc_gpu_run.  Calling it again replaces the set in place: it first waits
 * for all work on the device (hipDeviceSynchronize), so launches already
 * queued keep the parameters they were launched with.  States and host
 * pipelines are not affected (they hold their own copy).  Not to be called
 * concurrently with launches on the same device (see the top of this file). */
int cloudsc_gpu_init(int device, const cloudsc_params_t *params);

/* Enqueue one CLOUDSC step over ngptot columns on `stream` (a hipStream_t, or
 * NULL for the default stream) of `device`.  Asynchronous; errors in the launch
 * configuration are returned, asynchronous faults surface at the caller's sync.
 * SCC and KSEG need a workspace: pass scratch of cloudsc_gpu_scratch_bytes()
 * (KCACHE and SCC_PRIVATE need none: the latter's temporaries are the
 * kernel's private segment, sized by the HIP runtime at launch)
 * bytes (NULL is fine for KCACHE).  The KSEG workspace holds a dequeue counter
 * and per-block flags that are re-zeroed on `stream` before every launch, so one
 * workspace must not be shared by launches in flight on different streams.
 * nproma: 1..256 for KCACHE and SCC (one workgroup of nproma threads per
 * block), 1..2^24 for KSEG (64-column sub-blocks; all index arithmetic is
 * 64-bit); otherwise CLOUDSC_EINVAL.
 * A caller-owned KSEG workspace carries a sticky error word (below): zero it,
 * or pass it through cloudsc_gpu_check, before reusing the memory for a new
 * series of launches, or a stale count may surface as CLOUDSC_EHANDOFF. */
int cloudsc_gpu_run(int device, void *stream, int precision, int variant,
                    int ngptot, int nproma, int klev,
                    const cloudsc_fields_t *device_fields, void *scratch);

/* ------------------------------------------------------------------------ */
/* Caller-owned device fields, placed (round 5)                              */
/* ------------------------------------------------------------------------ */
/* How fast the kernel writes its 21 output fields depends on where they land
 * in HBM: field sets of one configuration ran the fp64 KSEG kernel at
 * 1.63-1.94 ms, and the slow ones stall on DRAM write credits (DESIGN.md
 * §3.12).  A placement search allocates candidate buffers, times a probe over
 * them and keeps a candidate when the probe is > 1 % faster.  Its cost and
 * result: */
typedef struct cloudsc_placement {
  float probe_first_ms, probe_final_ms;   /* probe time of the first / the kept placement            */
  int tries, moves;                       /* candidate buffers allocated / kept                      */
  int launches;                           /* probe launches run (untimed warm-ups included)          */
  int method;                             /* CLOUDSC_PLACE_METHOD_*                                  */
  double search_ms;                       /* wall time of the search                                 */
  long long peak_transient_bytes;         /* most device bytes held at once beyond the fields' own   */
  long long transient_budget_bytes;       /* the bound the free-memory check was made for (round 6):  */
                                          /* peak_transient_bytes never exceeds it; 0 = no search    */
} cloudsc_placement_t;
#define CLOUDSC_PLACE_METHOD_NONE        0   /* no search                                             */
#define CLOUDSC_PLACE_METHOD_KERNEL      1   /* the KSEG kernel on the state's own inputs (state API)  */
#define CLOUDSC_PLACE_METHOD_WRITE_PROBE 2   /* the kernel's output write pattern, no physics (round 5) */
#define CLOUDSC_PLACE_METHOD_RW_PROBE    3   /* the kernel's read + write pattern, no physics (round 6) */

/* cloudsc_fields_alloc flags */
#define CLOUDSC_PLACE_NONE     1   /* one allocation per field, no search (a caller that runs one step) */
#define CLOUDSC_ALLOC_AEROSOLS 2   /* also allocate the five aerosol inputs (LAERICESED/LAERICEAUTO)     */

/* Allocate the device buffers of every field of an (ngptot, nproma, klev,
 * precision) problem on `device` -- one allocation per field, block layout, as
 * the reference GPU driver's cudaMalloc calls do (cloudsc_driver.cu:276-328) --
 * for the caller to fill and to run with cloudsc_gpu_run.  Unless flags has
 * CLOUDSC_PLACE_NONE, the output buffers (plude included) are then placed by a
 * search timed with the kernel's memory pattern over the set -- every input
 * read and every output written as the KSEG kernel does, no physics, so no
 * field contents are needed: the caller fills the inputs afterwards (round 6:
 * reads and write-through stores, ranking 10 placements at Spearman 0.99
 * against the kernel, profiles/r06/place_corr_sc1_fp64.jsonl) -- 8 whole fresh
 * output sets, then up to two passes of one field at a time
 * (csrc/cloudsc_place.hip).  The search overwrites nothing the caller owns.
 * Input buffers are never moved (their placement does not change the kernel
 * time).  `report` (may be NULL) receives the search's cost and result.  On an
 * error nothing stays allocated. */
int cloudsc_fields_alloc(int device, int precision, int ngptot, int nproma, int klev, int flags,
                         cloudsc_fields_t *fields, cloudsc_placement_t *report);

/* Free the buffers cloudsc_fields_alloc made and set their pointers to NULL.
 * Non-NULL pointers it did not make (on this device) are left alone and make
 * the call return CLOUDSC_EINVAL. */
int cloudsc_fields_free(int device, cloudsc_fields_t *fields);

/* Bytes of device scratch a variant needs for (ngptot, nproma, klev, precision); 0 for KCACHE. */
long long cloudsc_gpu_scratch_bytes(int precision, int variant, int ngptot, int nproma, int klev);

/* Wait for `stream` and report failures the kernels count on the device.
 * For KSEG: a segment whose predecessor did not hand over its carried state
 * within the spin bound gives up and counts itself in the workspace; its
 * columns are then wrong.  The count accumulates over the KSEG launches on
 * `scratch` until this call reads it (and clears it): CLOUDSC_EHANDOFF if it is
 * non-zero.  Callers of cloudsc_gpu_run with KSEG should call it after their
 * launches (the state and pipeline APIs do).  Other variants: only the sync. */
int cloudsc_gpu_check(int device, void *stream, int variant, void *scratch);

/* Diagnostic: the number of polls a KSEG consumer makes before it gives up
 * (default 2^24, restored by a negative value).  0 makes every hand-off fail
 * without polling -- used by the tests of the error path. */
int cloudsc_debug_set_kseg_spin_limit(long long limit);

/* Diagnostic: override the KSEG schedule for this process -- nseg level
 * segments per column (1..16) and a grid of `grid` workgroups -- 0 restores
 * the measured default (2 guided segments, one workgroup per resident slot).
 * The result bits do not depend on either; the tests use it to exercise the
 * hand-offs with few workgroups and many segments. */
int cloudsc_debug_set_kseg_schedule(int nseg, int grid);

/* Diagnostic: field placement of the states created after this call.  < 0 (the
 * default): one device allocation per field.  >= 0: all fields of a state in
 * one allocation, field i starting at a 2 MiB boundary plus (i * stagger) mod
 * 2 MiB -- for measuring how the HBM placement of the ~47 concurrently
 * streamed fields affects the kernel time (tools/ab_layout.py).  stagger must
 * be a multiple of 256 bytes (CLOUDSC_EINVAL otherwise) and is taken modulo
 * 2 MiB.  alloc_flags must be 0 (CLOUDSC_EINVAL otherwise): states created
 * after destroyed states whose fields were hipDeviceMallocContiguous
 * allocations computed wrong values -- in part the round-3 parameter-upload
 * race (fixed), in part a cause not found (profiles/r04/contiguous_alloc_hazard.txt);
 * the diagnostic build (-DCLOUDSC_DEBUG_KNOBS) admits the flags to reproduce it. */
int cloudsc_debug_set_state_layout(long long stagger, unsigned alloc_flags);

/* Diagnostic: the kernels' single-precision exp/pow on the device, element-wise
 * over n host values: which = 0 the float-internal expf (CLOUDSC_FP32 default),
 * 1 its powf(x, y), 2 the glibc-algorithm expf (CLOUDSC_FP32_EXACT_LIBM),
 * 3 its powf, 4 the fast kernels' division x / y (v_rcp_f32 + one correction),
 * 5 the exact kernels' division.  y is read for 1, 3, 4 and 5 only. */
int cloudsc_debug_fp32_libm(int device, int which, const float *x, const float *y, float *out, long long n);

/* Human-readable message for an error code; last HIP error string of this thread. */
const char *cloudsc_strerror(int code);
const char *cloudsc_last_hip_error(void);

/* Measurement: the achievable HBM bandwidth of this device, a STREAM copy
 * between two buffers of bytes / 2 (>= 1 MiB each; 2 x bytes / 2 moved per
 * launch) in 16-byte-per-lane tiles, over three such buffer pairs allocated
 * together (their placement moves the rate by ~5 %), `reps` launches of each
 * tile shape per pair after one warm-up; the best launch, in GB/s (10^9 B/s).
 * bench.py reports it as roofline.achievable_peak beside the 8 TB/s spec. */
int cloudsc_hbm_copy_gbps(int device, long long bytes, int reps, double *gbps);

/* Measurement: the host<->device copy ceiling of this device, the bound of the
 * host-buffer pipeline: `bytes` (>= 1 MiB) of pinned host memory each way, one
 * stream per direction, 64 MiB copies; *h2d and *d2h one direction alone,
 * *both the total of the two directions copied at once; GB/s, best of `reps`.
 * bench.py reports pcie_inclusive against it. */
int cloudsc_pcie_gbps(int device, long long bytes, int reps, double *h2d, double *d2h, double *both);

/* Measurement: stream `bytes` (>= 1 MiB, a multiple of 16) through one device
 * buffer with `width` (4, 8 or 16) bytes per lane per access, non-temporal,
 * consecutive lanes on consecutive elements -- the CLOUDSC kernels' access
 * shape at width 8 (fp64) and 4 (fp32) -- as a read (mode 0) or a write
 * (mode 1); *ms = the fastest of `reps` launches.  A rocprofv3 PMC pass over it
 * calibrates FETCH_SIZE / WRITE_SIZE for those widths (tools/calib_counters.py). */
int cloudsc_debug_stream_probe(int device, int mode, int width, long long bytes, int reps, double *ms);

/* ABI introspection for bindings: sizeof of the public structs
 * (0 params, 1 fields, 2 template, 3 reference, 4 stats), -1 otherwise. */
long long cloudsc_abi_sizeof(int which);

/* ------------------------------------------------------------------------ */
/* CPU variant (BASELINE.json config 1): explicitly selected, never a fallback */
/* ------------------------------------------------------------------------ */

/* One CLOUDSC step over ngptot columns in HOST memory (block layout, fp64),
 * on `nthreads` host threads (<= 0: all hardware threads) taking NPROMA blocks
 * from a shared counter -- the C dwarf's OpenMP block loop
 * (src/cloudsc_c/cloudsc/cloudsc_driver.c:183-217) around the kernel
 * cloudsc_c() (cloudsc_c.c:19-2587).  The per-level physics is the same source
 * the GPU kernels are built from, compiled for the host; the output is the
 * reference kernel's bit for bit.  Same output contract as cloudsc_gpu_run
 * (every output element written, plude read-modify-write).  *seconds (may be
 * NULL) = wall time of the block loop.  Needs no GPU. */
int cloudsc_cpu_run(int nthreads, int ngptot, int nproma, int klev, const cloudsc_params_t *params,
                    const cloudsc_fields_t *host_fields, double *seconds);

/* cloudsc_cpu_run with the C dwarf's per-thread record (zinfo,
 * cloudsc_driver.c:185-228, printed as the "@ core#" rows at :238-253): for
 * thread t < nthreads, thread_seconds[t] = its wall time, thread_blocks[t] =
 * NPROMA blocks it took (icalls), thread_columns[t] = columns it computed
 * (igpc).  Each array (may be NULL) holds nthreads entries; nthreads must be
 * > 0 here.  Threads beyond the block count report zeros. */
int cloudsc_cpu_run_threads(int nthreads, int ngptot, int nproma, int klev, const cloudsc_params_t *params,
                            const cloudsc_fields_t *host_fields, double *seconds, double *thread_seconds,
                            int *thread_blocks, int *thread_columns);

/* ------------------------------------------------------------------------ */
/* Dwarf plumbing on the device: expand a KLON-column template to NGPTOT      */
/* columns (global column g -> template column g % klon, load_state.c:69-184, */
/* expand_mod.F90:173-200), run, time, and validate against a KLON-column     */
/* reference with the Fortran ERROR_PRINT statistics (validate_mod.F90:263). */
/* ------------------------------------------------------------------------ */

/* Template / reference arrays in the HDF5 / Serialbox order: [lev][klon],
 * species [nclv][lev][klon], surface [klon].  Always double (fp32 runs convert
 * at expansion, as file_io_mod.F90:96-112 does). */
typedef struct cloudsc_template {
  int klon, klev;
  const double *pt, *pq, *tendency_tmp_t, *tendency_tmp_q, *tendency_tmp_a, *tendency_tmp_cld;
  const double *pvfl, *pvfi, *phrsw, *phrlw, *pvervel, *pap, *paph, *plsm;
  const int    *ktype;
  const double *plu, *plude, *psnde, *pmfu, *pmfd, *pa, *pclv, *psupsat;
  const double *plcrit_aer, *picrit_aer, *pre_ice, *pccn, *pnice;   /* may be NULL */
} cloudsc_template_t;

/* The 21 validated fields, in the dwarf's print order (cloudsc_validate.c:193-216). */
#define CLOUDSC_NVALID 21
enum cloudsc_field_id {
  CLOUDSC_F_PLUDE = 0, CLOUDSC_F_PCOVPTOT, CLOUDSC_F_PRAINFRAC_TOPRFZ,
  CLOUDSC_F_PFSQLF, CLOUDSC_F_PFSQIF, CLOUDSC_F_PFCQLNG, CLOUDSC_F_PFCQNNG,
  CLOUDSC_F_PFSQRF, CLOUDSC_F_PFSQSF, CLOUDSC_F_PFCQRNG, CLOUDSC_F_PFCQSNG,
  CLOUDSC_F_PFSQLTUR, CLOUDSC_F_PFSQITUR, CLOUDSC_F_PFPLSL, CLOUDSC_F_PFPLSN,
  CLOUDSC_F_PFHPSL, CLOUDSC_F_PFHPSN, CLOUDSC_F_TENDENCY_LOC_A,
  CLOUDSC_F_TENDENCY_LOC_Q, CLOUDSC_F_TENDENCY_LOC_T, CLOUDSC_F_TENDENCY_LOC_CLD
};

/* Reference outputs for the KLON template columns, same order as the enum;
 * each array in template order ([lev][klon], [nclv][lev][klon] or [klon]). */
typedef struct cloudsc_reference {
  int klon, klev;
  const double *field[CLOUDSC_NVALID];
} cloudsc_reference_t;

/* Per-field statistics, the inputs of ERROR_PRINT (validate_mod.F90:263-296).
 * The two sums are carried as double-doubles: errsum / refsum are the sums
 * rounded to double, errsum_lo / refsum_lo what that rounding left over (all
 * terms are non-negative, so hi + lo holds the sum to ~100 bits).  Sums of
 * partial statistics -- NPROMA blocks on the device, shards on the host, the
 * MPI_Reduce of validate_mod.F90:53-55 -- therefore depend on how the columns
 * were partitioned only within the double-double error (~2^-100 relative): in
 * practice a sharded run prints the unsharded run's table to the last digit; a
 * total within that distance of a rounding midpoint could round 1 ulp apart.
 * Combine partials with cloudsc_stats_combine. */
typedef struct cloudsc_stats {
  double minval, maxval, maxerr, errsum, refsum;
  double errsum_lo, refsum_lo;
} cloudsc_stats_t;

/* acc <- acc (+) part: min of mins, max of maxes and of max|d|, double-double
 * sums.  Start from {DBL_MAX, -DBL_MAX, 0, 0, 0, 0, 0}. */
void cloudsc_stats_combine(cloudsc_stats_t *acc, const cloudsc_stats_t *part);

typedef struct cloudsc_gpu_state cloudsc_gpu_state_t;

/* Allocate device buffers for columns [col_offset, col_offset+ngptot) of the
 * global problem and expand the template into them on the device (g % klon
 * with g the GLOBAL column index, so a sharded run is bit-identical to an
 * unsharded one).  Keeps a pristine copy of plude for repeated runs. */
int cloudsc_state_create(cloudsc_gpu_state_t **state, int device, int precision,
                         int ngptot, int nproma, long long col_offset,
                         const cloudsc_template_t *tmpl, const cloudsc_params_t *params);

/* Device pointers of the state's buffers (block layout) -- for callers that
 * want to drive cloudsc_gpu_run themselves (cloudsc_gpu_run uses the device's
 * default parameter set, not the state's). */
int cloudsc_state_fields(const cloudsc_gpu_state_t *state, cloudsc_fields_t *out);

/* How the state's output fields were placed (round 4).  The rate at which
 * the kernel writes its 21 output fields depends on where they land in HBM
 * (fp64 KSEG 1.63-1.94 ms for states of one configuration: fields written
 * together whose physical pages collide stall on DRAM write credits).  At
 * creation the state times the KSEG kernel on its own inputs over candidate
 * placements of its outputs -- eight whole fresh output sets (the last seven
 * shuffled with spacers), then one field at a time -- then of its inputs
 * (four whole fresh input sets, the last three shuffled with spacers,
 * contents copied), and keeps a candidate when the time drops by more than
 * 1 %.  Each rejected input set is freed as soon as it loses.
 * If the search's launches time out in a segment hand-off, the first
 * placement is kept and probe_final_ms is negative (the state is created).
 * probe_first_ms / probe_final_ms: the kernel time of the first / the kept
 * placement, tries / moves: buffers (outputs and inputs) allocated as
 * candidates / kept.  Cost (wall time, launches, transient bytes):
 * cloudsc_state_placement_report.
 * All zero when the search was off.  Any pointer may be NULL. */
int cloudsc_state_placement(const cloudsc_gpu_state_t *state, float *probe_first_ms, float *probe_final_ms,
                            int *tries, int *moves);

/* The placement search of the state (cloudsc_state_placement) with its cost:
 * all of it, outputs and inputs, method CLOUDSC_PLACE_METHOD_KERNEL, or
 * CLOUDSC_PLACE_METHOD_NONE with zeros when the search was off. */
int cloudsc_state_placement_report(const cloudsc_gpu_state_t *state, cloudsc_placement_t *report);

/* Passes of the output placement search of the states created after this
 * call, process-wide (0 = off: the first allocation is kept; negative = the
 * default, 2; at most 8).  The results do not depend on it; the search costs
 * ~0.5 s of kernel launches per fp64 state at NGPTOT=163840 and pays off only
 * over many steps (the CLI turns it off for one step). */
int cloudsc_set_placement_search(int passes);
/* The same (the name of rounds 3-4). */
int cloudsc_debug_set_placement_search(int passes);

/* Measurement: the memory-pattern probe (csrc/cloudsc_place.hip) over the
 * device fields f: one wave per 64-column sub-block streams the level planes
 * the way the KSEG kernel does, with no physics.  mode 0 writes every non-NULL
 * output field; mode 1 also reads every input field.  *ms = best of `reps`
 * timed launches after one untimed.  Outputs (plude included) are
 * overwritten with junk; input contents do not matter.  It ranks placements
 * of a field set without its contents (tools/place_corr.py). */
int cloudsc_debug_memory_probe(int device, int precision, int ngptot, int nproma, int klev,
                               const cloudsc_fields_t *f, int mode, int reps, float *ms);

/* Diagnostic (round 6 layout study, tools/layout_corr.py): the same probe over
 * fields in another HBM layout.  strides[6] = the element strides between
 * blocks, between rows (levels) and between species planes of the inputs, then
 * of the outputs; 0 keeps the reference block layout's.  Each field pointer
 * addresses row 0 of block 0 (species 0) of its field; every element the
 * strides address must lie inside that field's allocation. */
int cloudsc_debug_memory_probe_layout(int device, int precision, int ngptot, int nproma, int klev,
                                      const cloudsc_fields_t *f, int mode, int reps, const long long *strides,
                                      float *ms);

/* Diagnostic, diagnostic build only (-DCLOUDSC_DEBUG_CANARY; otherwise
 * CLOUDSC_EINVAL): every device buffer of the states and placement searches
 * carries a 64 KiB guard band of a known byte on each side.  *live = guarded
 * buffers alive, *bad_allocs = those with a changed guard byte, *bad_bytes =
 * changed guard bytes in them plus those found when buffers were freed since
 * the last call.  For the round-5 record of the contiguous-allocation failure
 * (tools/contig_diag_r05.py). */
int cloudsc_debug_canary_check(int *live, int *bad_allocs, long long *bad_bytes);

/* Diagnostic: copy `bytes` (a multiple of 4) from device memory src to dst
 * with a kernel (4-byte vector loads and stores through the caches, a grid
 * over all XCDs), then wait -- to compare what the shader cores read with what
 * a copy engine (hipMemcpy) reads from the same memory. */
int cloudsc_debug_kernel_copy(void *dst, const void *src, long long bytes);

/* Diagnostic: move field `member` (its position in cloudsc_fields_t) of a state
 * to a new device allocation, contents copied; the old allocation is kept until
 * the state is destroyed, so the field lands on other physical pages.  For
 * finding which fields' placement decides the kernel time
 * (tools/placement_fields.py).  CLOUDSC_EINVAL for a member the state does not
 * hold (aerosol fields it was created without). */
int cloudsc_debug_state_relocate_field(cloudsc_gpu_state_t *s, int member);

/* Diagnostic: the same for a state buffer that is not a field: which = 0 the
 * pristine plude copy, 1 the KSEG workspace (zeroed again before the next
 * launch), 2 the SCC temporaries.  CLOUDSC_EINVAL when the state does not hold
 * it yet (workspaces are allocated on first use). */
int cloudsc_debug_state_relocate_aux(cloudsc_gpu_state_t *s, int which);

/* Restore plude from the pristine copy -- for callers that run in place
 * through cloudsc_gpu_run on the state's buffers. */
int cloudsc_state_reset(cloudsc_gpu_state_t *state);

/* Launch `reps` back-to-back steps of `variant` on the state's stream and
 * time each with HIP events recorded on that stream, with the state's own
 * parameter set.  The INOUT field plude
 * is taken out of place: every step reads the pristine input copy and writes
 * its result to the state's plude buffer, so repeated steps compute the same
 * step without a restore copy.  ms_per_step[reps] receives the per-step
 * kernel time, recorded by each launch's own dispatch (may be NULL: then no
 * events are recorded).  KSEG: CLOUDSC_EHANDOFF if a segment hand-off
 * timed out (cloudsc_gpu_check). */
int cloudsc_state_run(cloudsc_gpu_state_t *state, int variant, int reps, float *ms_per_step);

/* As cloudsc_state_run, timed as a whole: `reps` plain dispatches back to
 * back between two events on the state's stream; *span_ms = the time from the
 * first launch's start to the last one's end.  A dispatch that records its own
 * events (cloudsc_state_run with ms_per_step) leaves ~5 us more between
 * kernels than a plain one; span_ms / reps is the sustained time per step. */
int cloudsc_state_run_span(cloudsc_gpu_state_t *state, int variant, int reps, float *span_ms);

/* Wait for all work of the state's stream. */
int cloudsc_state_sync(cloudsc_gpu_state_t *state);

/* Measurement: the effective shader clock of the state's KSEG launches since
 * the last reset, in GHz -- every workgroup adds the shader-clock cycles
 * (s_memtime) and the 100 MHz real-time ticks (s_memrealtime) it spent in the
 * kernel to two counters in the KSEG workspace; *ghz = cycles / ticks x the
 * real-time rate (0 before any KSEG launch).  Waits for the state's stream;
 * reset != 0 zeroes the counters afterwards.  bench.py reports it beside the
 * kernel time (the fp64 kernel follows the board's clock). */
int cloudsc_state_kseg_clock(cloudsc_gpu_state_t *state, int reset, double *ghz);

/* Field-wise statistics vs a KLON-column reference, computed on the device
 * (modulo indexing; no expanded reference in host or device memory). */
int cloudsc_state_validate(cloudsc_gpu_state_t *state, const cloudsc_reference_t *ref,
                           cloudsc_stats_t stats[CLOUDSC_NVALID]);

/* Copy one validated output field to host memory in BLOCK layout as doubles
 * (fp32 states are widened).  `host` must hold the field's blocked size. */
int cloudsc_state_download(cloudsc_gpu_state_t *state, int field_id, double *host);

/* Element count of a validated field in block layout for this state. */
long long cloudsc_state_field_elems(const cloudsc_gpu_state_t *state, int field_id);

int cloudsc_state_destroy(cloudsc_gpu_state_t *state);

/* ------------------------------------------------------------------------ */
/* Host-buffer pipeline: the reference GPU drivers' H2D -> kernel -> D2H      */
/* (cloudsc_driver.cu:344-456), chunked and overlapped across streams         */
/* ------------------------------------------------------------------------ */
typedef struct cloudsc_host_pipeline cloudsc_host_pipeline_t;

/* `host` holds HOST pointers in block layout (full NPROMA blocks, the
 * precision's element type, ktype int).  The arrays are pinned in place
 * (hipHostRegister) until destroy; device buffers for `nstreams` chunk slots of
 * `chunk_blocks` blocks each are allocated here (1..16; chunk c uses slot
 * c % nstreams).  cloudsc_gpu_init must have been called for the device; the
 * pipeline keeps a copy of the device's default parameter set as it is at
 * creation. */
int cloudsc_host_pipeline_create(cloudsc_host_pipeline_t **pipe, int device, int precision, int ngptot,
                                 int nproma, int klev, int chunk_blocks, int nstreams,
                                 const cloudsc_fields_t *host);

/* One step over all columns, pipelined over three streams: every H2D copy
 * (inputs, plude) on one, every kernel on a second, every D2H copy (outputs,
 * plude) on a third, ordered per chunk slot by events, so chunk c's inputs
 * move in while chunk c-1 computes and chunk c-2's outputs move out.  *ms =
 * elapsed time of the whole pipeline (transfers included), HIP events on the
 * null stream.  KSEG: CLOUDSC_EHANDOFF if a segment hand-off timed out in any
 * chunk. */
int cloudsc_host_pipeline_run(cloudsc_host_pipeline_t *pipe, int variant, double *ms);

int cloudsc_host_pipeline_destroy(cloudsc_host_pipeline_t *pipe);

/* Diagnostic: how the pipeline's host arrays are mapped for the device.
 * *n_arrays = the number of non-NULL host arrays; *n_not_one_mapping = how many
 * of them are NOT covered by a single pinned mapping from their first to their
 * last byte (hipPointerGetAttributes at both ends, device addresses exactly
 * bytes-1 apart).  0 is the invariant create establishes (merged page ranges,
 * each registered once). */
int cloudsc_debug_host_pipeline_mapping(const cloudsc_host_pipeline_t *pipe, int *n_arrays,
                                        int *n_not_one_mapping);

/* Diagnostic: 1 if [ptr, ptr+bytes) is currently pinned host memory reachable
 * by the device as one mapping, 0 if not (e.g. after the pipeline that pinned
 * it was destroyed). */
int cloudsc_debug_host_pinned(const void *ptr, long long bytes);

/* Diagnostic: how host pipeline steps run after this call move their data.
 * 1 (the default; negative restores it): every copy issued by the pipeline on
 * a copy engine of its own per direction (hsa_amd_memory_async_copy_on_engine,
 * engines chosen at creation), ordered with the kernels from the host -- the
 * runtime's own engine choice for hipMemcpyAsync lets both directions land on
 * one engine now and then, which serialises them (~1.7-3.3x slower steps,
 * profiles/r04/pipeline_engines.txt).  0: three HIP streams (one per
 * direction, one for the kernels) with the runtime's engine choice.  2: as 0,
 * with the outputs written back by a copy kernel through the pinned memory's
 * device address.  A pipeline whose engines could not be set up at creation
 * runs as 0.  CLOUDSC_EINVAL for other modes. */
int cloudsc_debug_set_pipeline_copy(int mode);

/* Diagnostic: the copy path a pipeline was set up with: *mode 1 with the
 * engine masks (hsa_amd_sdma_engine_id_t bits) it copies on per direction, or
 * 0 (HIP streams) with both masks 0.  Any output pointer may be NULL. */
int cloudsc_debug_host_pipeline_copy(const cloudsc_host_pipeline_t *pipe, int *mode, int *h2d_engine,
                                     int *d2h_engine);

/* Measurement: the time of one step's copies WITHOUT the kernels, on the same
 * copy engines, host arrays and device slots (every input H2D, every output
 * D2H, each direction back to back on its engine): the bound a step of this
 * pipeline is held against (bench.py's pcie_inclusive.bound_ms).  The host
 * OUTPUT arrays and plude receive the device slots' contents, not results:
 * run a step (with plude restored) before reading outputs again.
 * CLOUDSC_EINVAL when the pipeline has no copy engines (HIP-stream mode). */
int cloudsc_host_pipeline_copy_bound(cloudsc_host_pipeline_t *pipe, double *ms);

/* Diagnostic: the engine pair check a pipeline ran at creation (copy mode 1):
 * *overlap = time of 256 MiB each way at once / the slower direction alone
 * (1.0 = the directions fully concurrent, 2.0 = serialised) for the pair it
 * kept, *pairs_tried = engine pairs measured (the first pair under 1.3 is
 * kept, else the best of at most 6).  Both 0 in HIP-stream mode. */
int cloudsc_debug_host_pipeline_engine_check(const cloudsc_host_pipeline_t *pipe, double *overlap,
                                             int *pairs_tried);

/* ------------------------------------------------------------------------ */
/* One synchronous step on host arrays, callable from any host thread        */
/* ------------------------------------------------------------------------ */
/* The per-block call of the reference C dwarf's OpenMP loop
 * (src/cloudsc_c/cloudsc/cloudsc_driver.c:183-217 calls cloudsc_c() on one
 * NPROMA block from every thread) moved to the device: copy the inputs and
 * plude in (pageable memory is fine), run `variant`, copy the outputs and plude
 * back, wait.  `host` holds HOST pointers in block layout, like
 * cloudsc_cpu_run.  No cloudsc_gpu_init is needed: each calling thread keeps,
 * per device, its own stream, device buffers (grown to the largest call), KSEG
 * workspace and parameter set (uploaded again only when *params changes), so
 * concurrent callers share nothing.  Same output contract as cloudsc_gpu_run.
 * The drop-in cloudsc_c() of libcloudsc_c_amd_gpu.so (csrc/cloudsc_c_dropin.c)
 * is built on it. */
int cloudsc_host_run(int device, int precision, int variant, int ngptot, int nproma, int klev,
                     const cloudsc_params_t *params, const cloudsc_fields_t *host);

/* Free the calling thread's cloudsc_host_run contexts (device buffers, stream,
 * parameter sets) on every device; the next cloudsc_host_run creates them again. */
int cloudsc_host_run_release(void);

/* Where a cloudsc_host_run call's time goes (round 6, VERDICT r05 weak 6: the
 * GPU drop-in's per-call cost).  Sums over the calls of every thread since
 * profiling was enabled, in ms, each thread's FIRST call on a device left out
 * of them (it creates the thread's context and, in a fresh process, starts the
 * HIP runtime: first_calls / first_calls_ms count those apart): host side measured with a steady clock, the
 * device side with HIP events on the call's stream between its three
 * operations.  alloc: the calling thread's context, device selection, parameter
 * upload and buffer growth (the first calls: the HIP runtime's own start-up
 * lands here); setup: argument checks and the image layout; enqueue: issuing
 * the copies and the launch; pack / unpack: the active lanes between the caller's
 * arrays and the pinned staging buffer; h2d / kernel / d2h: the input copy, the
 * CLOUDSC launch (the KSEG prepare kernel included) and the output copy on the
 * device; wait: from the last enqueue to the stream sync's return (the device
 * work the host waits for); total: whole calls = alloc + setup + pack +
 * enqueue + wait + unpack. */
typedef struct cloudsc_host_run_profile {
  long long calls;
  double setup_ms, pack_ms, h2d_ms, kernel_ms, d2h_ms, wait_ms, unpack_ms, total_ms;
  double alloc_ms;     /* part of total_ms, not of setup_ms */
  double enqueue_ms;
  double max_call_ms;  /* the slowest single call counted */
  long long first_calls;
  double first_calls_ms;
} cloudsc_host_run_profile_t;
/* mode 1: zero the sums and start profiling (each call then records 4 events);
 * mode 0: copy the sums into *out (may be NULL) and keep profiling;
 * mode -1: copy the sums into *out (may be NULL) and stop. */
int cloudsc_host_run_profile(int mode, cloudsc_host_run_profile_t *out);

#ifdef __cplusplus
}
#endif
#endif /* CLOUDSC_AMD_H */
