/*
 * dwarf_cloudsc_amd.c -- the dwarf host driver for MI355X:
 *
 *   dwarf-cloudsc-amd <nthreads> <ngptot> <nproma> [options]
 *
 * Same CLI, flow and stdout format as the reference C dwarf
 * (src/cloudsc_c/dwarf_cloudsc.c:17-50, cloudsc_driver.c:33-263): load the
 * KLON-column state (load_state.c), expand it to NGPTOT columns in NPROMA
 * blocks, run CLOUDSC, print the timing table, validate the 21 output fields
 * against the reference (cloudsc_validate.c:186-216).  Differences, all on
 * purpose:
 *   - the kernel runs on the GPU(s) through libcloudsc_amd.so (include/
 *     cloudsc_amd.h); expansion and the validation statistics run on the
 *     device against the KLON-column reference with the g % klon map, so no
 *     NGPTOT-sized host arrays exist;
 *   - HDF5 files are opened read-only (load_state.c:60,499,746 open RDWR);
 *     without input.h5 the raw dataset (data/cloudsc100) is read;
 *   - validation uses fabs like the Fortran ERROR_PRINT (validate_mod.F90:
 *     263-296), not the C validator's integer abs (cloudsc_validate.c:74);
 *   - the TOTAL line's col/s is NGPTOT/time (cloudsc_driver.c:261 prints the
 *     last thread's value);
 *   - exit status 1 if any field's relative L1 error exceeds the gate
 *     (--tol; default in fp64 the dwarf's own '!!!!' line, 10*eps: the
 *     fp64 kernels reproduce the reference kernel bit for bit; fp32 is
 *     reported without a gate unless --tol is given);
 *   - --gpus N shards the columns over N devices (block-aligned contiguous
 *     ranges of the GLOBAL column index, one host thread + stream per shard,
 *     no collective); statistics are combined on the host like the
 *     MPI_Reduce of validate_mod.F90:53-55.  With fewer visible devices than
 *     shards, shard d runs on device d % ndev (the shards of one device then
 *     share it; results are the same bits, only the timing differs).
 *
 * nthreads is the host thread count of --variant cpu (the library's CPU
 * variant, BASELINE.json config 1: `1 16384 32`); for the GPU variants it is
 * accepted and printed as NUMOMP for compatibility, the host threads being
 * one per shard.
 */
#define _GNU_SOURCE
#include <float.h>
#include <limits.h>
#include <math.h>
#include <dirent.h>
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "cloudsc_amd.h"
#include "cloudsc_io.h"

#define ZHPM 12482329.0   /* HPM flop count for 100 columns (cloudsc_driver.c:101) */
#define VARIANT_CPU 0     /* --variant cpu: cloudsc_cpu_run on the host cores (config 1) */

typedef struct {
  int numomp, ngptot, nproma, ngpus, precision, variant, reps, warmup;
  int transfer, chunk_blocks, nstreams, exact_libm;
  int place;                      /* placement search: 1 on, 0 off, -1 auto (on when reps > 1) */
  double energy_s;                /* --energy: seconds of back-to-back launches sampled for board power */
  double tol;
  int tol_given;
  const char *input_h5, *reference_h5, *data_dir, *write_h5_dir;
} options_t;

typedef struct {
  int device, ngptot, nproma, precision, variant, reps, warmup;
  int libm_bit;                   /* CLOUDSC_FP32_EXACT_LIBM or 0 */
  double energy_s;
  long long col_offset;
  const cloudsc_template_t *tmpl;
  const cloudsc_params_t *params;
  const cloudsc_reference_t *ref;
  pthread_barrier_t *barrier;
  /* results */
  int rc;
  char err[256];                  /* this shard's cloudsc_last_hip_error() (thread-local in the library) */
  double t_start, t_end;          /* seconds, CLOCK_MONOTONIC */
  float *kernel_ms;
  cloudsc_placement_t place;      /* the state's placement search and its cost */
  char power_path[512];           /* the device's hwmon power file ("" = none) */
  double board_w, energy_ms_per_step;   /* mean board power over the energy window, and its time per launch */
  int power_samples, energy_steps;
  cloudsc_stats_t stats[CLOUDSC_NVALID];
} shard_t;

static const char *variant_name(int v) {
  switch (v) {
    case CLOUDSC_VARIANT_KSEG: return "kseg";
    case CLOUDSC_VARIANT_KCACHE: return "kcache";
    case CLOUDSC_VARIANT_SCC: return "scc";
    case CLOUDSC_VARIANT_SCC_PRIVATE: return "scc-private";
    default: return "cpu";
  }
}

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void usage(const char *prog) {
  fprintf(stderr,
          "usage: %s [<nthreads> <ngptot> <nproma>] [options]\n"
          "  --gpus N              shard the columns over N devices (default 1)\n"
          "  --precision fp64|fp32 (default fp64)\n"
          "  --variant kseg|kcache|scc|scc-private|cpu (default kseg; cpu = the library's CPU variant on\n"
          "                        <nthreads> host threads, host-memory fields: BASELINE config 1)\n"
          "  --fp32-exact-libm     fp32: exp/pow with the glibc algorithms (bit-identical to the fp32\n"
          "                        restatement) instead of the default float-internal device forms\n"
          "  --reps R              timed steps (default 1)\n"
          "  --place on|off|auto   output placement search at state creation (~0.5 s, ~250 kernel\n"
          "                        launches; default auto: on when --reps > 1, off for one step)\n"
          "  --warmup W            untimed steps before the timed ones (default 1)\n"
          "  --energy S            after the timed steps, S seconds of back-to-back launches with the\n"
          "                        device's board power sampled every 10 ms (hwmon power1_input):\n"
          "                        prints an ENERGY line per shard (uJ per column)\n"
          "  --input FILE          input HDF5 file (default ./input.h5 when present)\n"
          "  --reference FILE      reference HDF5 file (default ./reference.h5 when present)\n"
          "  --data DIR            raw dataset directory (default $CLOUDSC_DATA or the\n"
          "                        repository's data/cloudsc100)\n"
          "  --tol X               relative L1 gate per field (default 10*eps = 2.2e-15 for fp64)\n"
          "  --transfer            host-buffer path: block-layout arrays in host memory,\n"
          "                        H2D -> kernel -> D2H per chunk, overlapped on streams\n"
          "                        (TOTAL includes the transfers, like cloudsc_driver.cu)\n"
          "  --chunk B --streams S chunk size in NPROMA blocks (128) and device chunk slots (3)\n"
          "  --write-h5 DIR        write DIR/input.h5 and DIR/reference.h5 of the loaded\n"
          "                        dataset and exit\n",
          prog);
}

static int parse(int argc, char **argv, options_t *o) {
  memset(o, 0, sizeof(*o));
  o->numomp = 1; o->ngptot = 100; o->nproma = 4;     /* dwarf_cloudsc.c:25-27 defaults */
  o->ngpus = 1; o->precision = CLOUDSC_FP64; o->variant = CLOUDSC_VARIANT_KSEG;
  o->reps = 1; o->warmup = 1; o->tol = 10.0 * DBL_EPSILON; o->place = -1;
  o->chunk_blocks = 128; o->nstreams = 3;  /* chunk slots; profiles/r04/transfer_sweep_kseg_fp64.txt */
  int npos = 0;
  long pos[3] = {0, 0, 0};
  for (int i = 1; i < argc; i++) {
    const char *a = argv[i];
    const char *v = i + 1 < argc ? argv[i + 1] : NULL;
#define NEEDV() do { if (!v) { fprintf(stderr, "%s needs a value\n", a); return -1; } i++; } while (0)
    if (!strcmp(a, "--gpus")) { NEEDV(); o->ngpus = atoi(v); }
    else if (!strcmp(a, "--precision")) {
      NEEDV();
      if (!strcmp(v, "fp64") || !strcmp(v, "dp")) o->precision = CLOUDSC_FP64;
      else if (!strcmp(v, "fp32") || !strcmp(v, "sp")) o->precision = CLOUDSC_FP32;
      else { fprintf(stderr, "bad precision %s\n", v); return -1; }
    } else if (!strcmp(a, "--variant")) {
      NEEDV();
      if (!strcmp(v, "kseg")) o->variant = CLOUDSC_VARIANT_KSEG;
      else if (!strcmp(v, "kcache")) o->variant = CLOUDSC_VARIANT_KCACHE;
      else if (!strcmp(v, "scc")) o->variant = CLOUDSC_VARIANT_SCC;
      else if (!strcmp(v, "scc-private")) o->variant = CLOUDSC_VARIANT_SCC_PRIVATE;
      else if (!strcmp(v, "cpu")) o->variant = VARIANT_CPU;
      else { fprintf(stderr, "bad variant %s\n", v); return -1; }
    } else if (!strcmp(a, "--reps")) { NEEDV(); o->reps = atoi(v); }
    else if (!strcmp(a, "--warmup")) { NEEDV(); o->warmup = atoi(v); }
    else if (!strcmp(a, "--energy")) {
      NEEDV();
      char *end;
      o->energy_s = strtod(v, &end);
      if (*end || !(o->energy_s >= 0.0) || o->energy_s > 600.0) { fprintf(stderr, "bad --energy %s\n", v); return -1; }
    }
    else if (!strcmp(a, "--place")) {
      NEEDV();
      if (!strcmp(v, "on")) o->place = 1;
      else if (!strcmp(v, "off")) o->place = 0;
      else if (!strcmp(v, "auto")) o->place = -1;
      else { fprintf(stderr, "bad --place %s\n", v); return -1; }
    }
    else if (!strcmp(a, "--input")) { NEEDV(); o->input_h5 = v; }
    else if (!strcmp(a, "--reference")) { NEEDV(); o->reference_h5 = v; }
    else if (!strcmp(a, "--data")) { NEEDV(); o->data_dir = v; }
    else if (!strcmp(a, "--tol")) { NEEDV(); o->tol = atof(v); o->tol_given = 1; }
    else if (!strcmp(a, "--write-h5")) { NEEDV(); o->write_h5_dir = v; }
    else if (!strcmp(a, "--transfer")) o->transfer = 1;
    else if (!strcmp(a, "--fp32-exact-libm")) o->exact_libm = 1;
    else if (!strcmp(a, "--chunk")) { NEEDV(); o->chunk_blocks = atoi(v); }
    else if (!strcmp(a, "--streams")) { NEEDV(); o->nstreams = atoi(v); }
    else if (!strcmp(a, "-h") || !strcmp(a, "--help")) return -1;
    else if (a[0] == '-' && a[1] == '-') { fprintf(stderr, "unknown option %s\n", a); return -1; }
    else {
      if (npos >= 3) { fprintf(stderr, "too many arguments\n"); return -1; }
      char *end;
      pos[npos++] = strtol(a, &end, 10);
      if (*end) { fprintf(stderr, "not a number: %s\n", a); return -1; }
    }
#undef NEEDV
  }
  if (npos != 0 && npos != 3) {
    /* dwarf_cloudsc.c:45-48 */
    printf("Calling c-cloudsc with the right number of arguments will work better ;-) \n");
    return -1;
  }
  if (npos == 3) {
    o->numomp = (int)pos[0]; o->ngptot = (int)pos[1]; o->nproma = (int)pos[2];
    if (o->numomp <= 0) o->numomp = 1;
  }
  /* KCACHE/SCC run one workgroup of NPROMA threads per block; KSEG any NPROMA */
  const int max_nproma = (o->variant == CLOUDSC_VARIANT_KSEG || o->variant == VARIANT_CPU) ? (1 << 24) : 256;
  if (o->ngptot <= 0 || o->nproma <= 0 || o->nproma > max_nproma || o->ngpus <= 0 || o->reps <= 0 ||
      o->warmup < 0) {
    fprintf(stderr, "invalid sizes: ngptot %d nproma %d (1..%d) gpus %d reps %d\n", o->ngptot, o->nproma,
            max_nproma, o->ngpus, o->reps);
    return -1;
  }
  return 0;
}

/* the raw dataset next to the executable: <exe dir>/../data/cloudsc100 */
static void default_data_dir(char *out, size_t n) {
  const char *env = getenv("CLOUDSC_DATA");
  if (env && *env) { snprintf(out, n, "%s", env); return; }
  char exe[PATH_MAX - 64];
  ssize_t len = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
  if (len <= 0) { snprintf(out, n, "data/cloudsc100"); return; }
  exe[len] = 0;
  char *slash = strrchr(exe, '/');
  if (slash) *slash = 0;
  snprintf(out, n, "%s/../data/cloudsc100", exe);
}

static int exists(const char *p) { return access(p, R_OK) == 0; }

/* ---- board power (--energy): the reference reads energy beside its timings
 * (EC_PMON, src/common/module/ec_pmon_mod.F90, dwarf_cloudsc.F90:42-46).  On an
 * MI355X host the GPU's sensor is its hwmon power file in microwatts, found
 * through the device's PCI bus id (hipDeviceGetPCIBusId, from the HIP runtime
 * the library has loaded); read-only. ---- */
static void power_file(int device, char *out, size_t n) {
  out[0] = 0;
  void *hip = dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
  if (!hip) hip = dlopen("libamdhip64.so", RTLD_NOW);
  if (!hip) return;
  int (*bus_id)(char *, int, int) = (int (*)(char *, int, int))dlsym(hip, "hipDeviceGetPCIBusId");
  char bus[64];
  if (!bus_id || bus_id(bus, (int)sizeof(bus), device) != 0) return;
  for (char *c = bus; *c; c++)
    if (*c >= 'A' && *c <= 'F') *c = (char)(*c - 'A' + 'a');
  char dir[256];
  snprintf(dir, sizeof(dir), "/sys/bus/pci/devices/%s/hwmon", bus);
  DIR *d = opendir(dir);
  if (!d) return;
  struct dirent *e;
  while ((e = readdir(d))) {
    if (strncmp(e->d_name, "hwmon", 5)) continue;
    static const char *names[2] = {"power1_input", "power1_average"};
    for (int k = 0; k < 2 && !out[0]; k++) {
      char f[512];
      snprintf(f, sizeof(f), "%.256s/%.64s/%.32s", dir, e->d_name, names[k]);
      FILE *fp = fopen(f, "r");
      if (!fp) continue;
      long long uw;
      if (fscanf(fp, "%lld", &uw) == 1) snprintf(out, n, "%s", f);
      fclose(fp);
    }
    if (out[0]) break;
  }
  closedir(d);
}

typedef struct {
  const char *path;
  volatile int stop;
  double sum_w;
  int n;
} sampler_t;

static void *sampler_main(void *arg) {
  sampler_t *sp = (sampler_t *)arg;
  const struct timespec period = {0, 10 * 1000 * 1000};
  while (!sp->stop) {
    FILE *fp = fopen(sp->path, "r");
    if (fp) {
      long long uw;
      if (fscanf(fp, "%lld", &uw) == 1) { sp->sum_w += uw * 1e-6; sp->n++; }
      fclose(fp);
    }
    nanosleep(&period, NULL);
  }
  return NULL;
}

/* S seconds of back-to-back launches (plain dispatches, timed 20 at a time) with
 * the board power sampled: mean W and the time per launch, for the ENERGY line */
static int energy_window(shard_t *s, cloudsc_gpu_state_t *st) {
  power_file(s->device, s->power_path, sizeof(s->power_path));
  if (!s->power_path[0]) return CLOUDSC_OK;
  sampler_t sp = {s->power_path, 0, 0.0, 0};
  pthread_t th;
  if (pthread_create(&th, NULL, sampler_main, &sp)) return CLOUDSC_OK;
  const double t0 = now();
  double span_ms = 0.0;
  int steps = 0, rc = CLOUDSC_OK;
  while (!rc && now() - t0 < s->energy_s) {
    float ms = 0.f;
    rc = cloudsc_state_run_span(st, s->variant | s->libm_bit, 20, &ms);
    span_ms += ms;
    steps += 20;
  }
  sp.stop = 1;
  pthread_join(th, NULL);
  s->power_samples = sp.n;
  s->board_w = sp.n ? sp.sum_w / sp.n : 0.0;
  s->energy_steps = steps;
  s->energy_ms_per_step = steps ? span_ms / steps : 0.0;
  return rc;
}

static void *shard_main(void *arg) {
  shard_t *s = (shard_t *)arg;
  cloudsc_gpu_state_t *st = NULL;
  s->rc = cloudsc_state_create(&st, s->device, s->precision, s->ngptot, s->nproma, s->col_offset, s->tmpl,
                               s->params);
  if (!s->rc) s->rc = cloudsc_state_placement_report(st, &s->place);
  if (!s->rc && s->warmup > 0) {
    float *w = (float *)malloc(sizeof(float) * s->warmup);
    s->rc = w ? cloudsc_state_run(st, s->variant | s->libm_bit, s->warmup, w) : CLOUDSC_ENOMEM;
    free(w);
  }
  if (!s->rc) s->rc = cloudsc_state_sync(st);
  /* every shard reaches the barrier, also after an error, so nobody waits forever */
  pthread_barrier_wait(s->barrier);
  s->t_start = now();
  if (!s->rc) s->rc = cloudsc_state_run(st, s->variant | s->libm_bit, s->reps, s->kernel_ms);
  if (!s->rc) s->rc = cloudsc_state_sync(st);
  s->t_end = now();
  pthread_barrier_wait(s->barrier);
  /* untimed; every launch is the same step (plude is taken out of place), so
   * the validation below still checks the timed step's results */
  if (!s->rc && s->energy_s > 0.0) s->rc = energy_window(s, st);
  if (!s->rc && s->ref) s->rc = cloudsc_state_validate(st, s->ref, s->stats);
  if (s->rc) snprintf(s->err, sizeof(s->err), "%s", cloudsc_last_hip_error());
  if (st) cloudsc_state_destroy(st);
  return NULL;
}

/* ERROR_PRINT (validate_mod.F90:263-296 / cloudsc_validate.c:20-44) */
static double print_error(const char *name, int ndim, const cloudsc_stats_t *s, int ngptot) {
  const double eps = DBL_EPSILON;
  double rel;
  int iopt;
  if (s->errsum < eps) { rel = 0.0; iopt = 1; }
  else if (s->refsum < eps) { rel = s->errsum / (1.0 + s->refsum); iopt = 2; }
  else { rel = s->errsum / s->refsum; iopt = 3; }
  printf(" %20s %dD%d %20.13le %20.13le %20.13le %20.13le %20.13le %s\n", name, ndim, iopt, s->minval, s->maxval,
         s->maxerr, s->errsum / (double)ngptot, 100.0 * rel, rel > 10.0 * eps ? " !!!!" : "     ");
  return rel;
}

/* ---- host-memory paths: --transfer (GPU, H2D/D2H per chunk) and --variant cpu ---- */
/* cloudsc_io input index -> cloudsc_fields_t member index */
static int input_field_index(int i) {
  if (i < 16) return i;                 /* pt .. plu */
  if (i == 16) return 27;               /* plude (INOUT) */
  if (i < 23) return i - 1;             /* psnde .. psupsat */
  return i - 1;                         /* aerosols 22..26 */
}
/* validated field id -> cloudsc_fields_t member index */
static const int k_valid_field[CLOUDSC_NVALID] = {27, 32, 33, 34, 35, 37, 36, 38, 39, 40, 41,
                                                  42, 43, 44, 45, 46, 47, 30, 29, 28, 31};
/* kinds of the outputs 28..47 */
static const int k_out_kind[20] = {0, 0, 0, 2, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};

static double print_error(const char *name, int ndim, const cloudsc_stats_t *s, int ngptot);

static int run_host(const options_t *o, const cloudsc_dataset_t *ds) {
  const int cpu = o->variant == VARIANT_CPU;
  const int es = o->precision == CLOUDSC_FP64 ? 8 : 4;
  const int nb = o->ngptot / o->nproma + (o->ngptot % o->nproma ? 1 : 0);
  const int aer = ds->params.laericesed || ds->params.laericeauto;
  cloudsc_fields_t f;
  memset(&f, 0, sizeof(f));
  void **fp = (void **)&f;
  size_t host_bytes = 0;
  double *plude0 = NULL;
  int rc = CLOUDSC_OK;
  /* inputs: expanded on the host (load_state.c) */
  for (int i = 0; i < CLOUDSC_IO_NIN && !rc; i++) {
    const int kind = cloudsc_io_input_kind[i];
    const void *src = i == CLOUDSC_IO_KTYPE ? (const void *)ds->ktype : (const void *)ds->in[i];
    if (!src || (i >= CLOUDSC_IO_FIRST_AEROSOL && !aer)) continue;
    const int is_int = i == CLOUDSC_IO_KTYPE;
    const size_t n = (size_t)nb * (size_t)(cloudsc_io_elems(kind, ds->klev, o->nproma));
    const size_t bytes = n * (is_int ? sizeof(int) : (size_t)es);
    void *dst = aligned_alloc(4096, (bytes + 4095) & ~(size_t)4095);
    if (!dst) { rc = CLOUDSC_ENOMEM; break; }
    cloudsc_io_expand(src, kind, is_int, ds->klev, ds->klon, o->ngptot, o->nproma, 0, is_int ? 4 : es, dst);
    fp[input_field_index(i)] = dst;
    host_bytes += bytes;
    if (i == 16) {
      plude0 = (double *)malloc(bytes);
      if (!plude0) { rc = CLOUDSC_ENOMEM; break; }
      memcpy(plude0, dst, bytes);
    }
  }
  for (int j = 0; j < 20 && !rc; j++) {
    const size_t bytes = (size_t)nb * (size_t)cloudsc_io_elems(k_out_kind[j], ds->klev, o->nproma) * es;
    void *dst = aligned_alloc(4096, (bytes + 4095) & ~(size_t)4095);
    if (!dst) { rc = CLOUDSC_ENOMEM; break; }
    memset(dst, 0xff, bytes);            /* NaN: the callee must write every element */
    fp[28 + j] = dst;
    host_bytes += bytes;
  }
  const size_t plude_bytes = (size_t)nb * ds->klev * o->nproma * es;
  cloudsc_host_pipeline_t *pipe = NULL;
  if (!rc && !cpu) rc = cloudsc_gpu_init(0, &ds->params);
  if (!rc && !cpu) rc = cloudsc_host_pipeline_create(&pipe, 0, o->precision, o->ngptot, o->nproma, ds->klev,
                                                     o->chunk_blocks, o->nstreams, &f);
  double total_ms = 0.0;
  /* --variant cpu: the per-thread record of the C dwarf (zinfo), summed over the timed steps */
  const int nth = o->numomp;
  double *th_s = cpu ? (double *)calloc((size_t)nth, sizeof(double)) : NULL;
  double *th_step = cpu ? (double *)calloc((size_t)nth, sizeof(double)) : NULL;
  int *th_blk = cpu ? (int *)calloc((size_t)nth, sizeof(int)) : NULL;
  int *th_col = cpu ? (int *)calloc((size_t)nth, sizeof(int)) : NULL;
  int *th_blk_step = cpu ? (int *)calloc((size_t)nth, sizeof(int)) : NULL;
  int *th_col_step = cpu ? (int *)calloc((size_t)nth, sizeof(int)) : NULL;
  if (cpu && (!th_s || !th_step || !th_blk || !th_col || !th_blk_step || !th_col_step)) rc = CLOUDSC_ENOMEM;
  for (int r = 0; r < o->warmup + o->reps && !rc; r++) {
    memcpy(f.plude, plude0, plude_bytes);                 /* INOUT restored, outside the timing */
    double ms = 0.0;
    if (cpu) {
      double secs = 0.0;
      rc = cloudsc_cpu_run_threads(nth, o->ngptot, o->nproma, ds->klev, &ds->params, &f, &secs, th_step,
                                   th_blk_step, th_col_step);
      ms = 1e3 * secs;
      if (r >= o->warmup)
        for (int t = 0; t < nth; t++) { th_s[t] += th_step[t]; th_blk[t] += th_blk_step[t]; th_col[t] += th_col_step[t]; }
    } else {
      rc = cloudsc_host_pipeline_run(pipe, o->variant | (o->exact_libm ? CLOUDSC_FP32_EXACT_LIBM : 0), &ms);
    }
    if (r >= o->warmup) total_ms += ms;
  }
  if (pipe) cloudsc_host_pipeline_destroy(pipe);
  int bad = 0;
  if (!rc) {
    const double t = 1e-3 * total_ms;
    const double cols = (double)o->ngptot * o->reps;
    printf("     NUMOMP=%d, NGPTOT=%d, NPROMA=%d, NGPBLKS=%d\n", o->numomp, o->ngptot, o->nproma, nb);
    printf(" Reference MFLOP count for 100 columns : %12.8f\n", 1.0e-06 * ZHPM);
    printf(" %10s%10s%10s%10s%10s %4s : %10s%10s%10s\n", "NUMOMP", "NGPTOT", "#GP-cols", "#BLKS", "NPROMA",
           "tid#", "Time(msec)", "MFlops/s", "col/s");
    /* per-thread rows (cloudsc_driver.c:238-253): columns and blocks of the last
     * step; time, MFlops/s and col/s over all timed steps like the TOTAL row */
    for (int t = 0; cpu && t < nth; t++) {
      const double tl = th_s[t], zfrac = (double)th_col[t] / cols;
      printf(" %10d%10d%10d%10d%10d %4d : %10d%10d%10d @ core#\n", o->numomp, o->ngptot, th_col_step[t],
             th_blk_step[t], o->nproma, t, (int)(tl * 1000.),
             tl > 0 ? (int)(1.0e-06 * zfrac * ZHPM * (cols / 100.) / tl) : 0, tl > 0 ? (int)(cols / tl) : 0);
    }
    printf(" %10d%10d%10d%10d%10d %4d : %10d%10d%10d TOTAL\n", o->numomp, o->ngptot, o->ngptot, nb, o->nproma, -1,
           (int)(t * 1000.), (int)(1.0e-06 * ZHPM * (cols / 100.) / t), (int)(cols / t));
    if (cpu)
      printf(" TIMING: steps=%d cpu_ms_per_step=%.4f columns_per_s=%.1f host_bytes=%zu threads=%d "
             "(cloudsc_cpu_run, host cores)\n",
             o->reps, total_ms / o->reps, cols / t, host_bytes, o->numomp);
    else
      printf(" TIMING: steps=%d transfer_ms_per_step=%.4f columns_per_s=%.1f host_bytes=%zu chunk_blocks=%d "
             "streams=%d (H2D + kernel + D2H, pinned host memory)\n",
             o->reps, total_ms / o->reps, cols / t, host_bytes, o->chunk_blocks, o->nstreams);
    if (ds->has_reference) {
      printf(" %20s %s %20s %20s %20s %20s %20s\n", "Variable", "Dim", "MinValue", "MaxValue", "AbsMaxErr",
             "AvgAbsErr/GP", "MaxRelErr-%");
      const int gate = o->precision == CLOUDSC_FP64 || o->tol_given;
      double worst = 0.0;
      for (int v = 0; v < CLOUDSC_NVALID; v++) {
        cloudsc_stats_t st;
        const int kind = cloudsc_io_ref_kind[v];
        cloudsc_io_field_stats(ds->ref[v], kind, ds->klev, ds->klon, fp[k_valid_field[v]], es, o->ngptot,
                               o->nproma, 0, &st);
        const double rel = print_error(cloudsc_io_print_names[v], kind == 3 ? 1 : kind == 2 ? 3 : 2, &st,
                                       o->ngptot);
        if (rel > worst) worst = rel;
        if (gate && !(rel <= o->tol)) bad++;
      }
      if (gate)
        printf(" VALIDATION: %s (worst relative L1 error %.3e, gate %.1e, %d field(s) over)\n",
               bad ? "FAILED" : "PASSED", worst, o->tol, bad);
      else
        printf(" VALIDATION: reported only (fp32 vs the fp64 reference; worst relative L1 error %.3e)\n", worst);
    }
  } else {
    fprintf(stderr, "dwarf-cloudsc-amd %s: %s (%s)\n", cpu ? "--variant cpu" : "--transfer", cloudsc_strerror(rc),
            cloudsc_last_hip_error());
  }
  for (int i = 0; i < 48; i++) free(fp[i]);
  free(plude0);
  free(th_s); free(th_step); free(th_blk); free(th_col); free(th_blk_step); free(th_col_step);
  return rc ? EXIT_FAILURE : (bad ? EXIT_FAILURE : EXIT_SUCCESS);
}

int main(int argc, char **argv) {
  options_t o;
  if (parse(argc, argv, &o)) { usage(argv[0]); return EXIT_FAILURE; }

  /* ---- load the KLON-column state (HDF5 read-only, else raw) ---- */
  cloudsc_dataset_t ds;
  int rc;
  const char *in_h5 = o.input_h5 ? o.input_h5 : (exists("input.h5") ? "input.h5" : NULL);
  if (in_h5) {
    const char *ref_h5 = o.reference_h5 ? o.reference_h5 : (exists("reference.h5") ? "reference.h5" : NULL);
    rc = cloudsc_io_load_hdf5(in_h5, ref_h5, &ds);
  } else {
    char dir[PATH_MAX];
    if (o.data_dir) snprintf(dir, sizeof(dir), "%s", o.data_dir);
    else default_data_dir(dir, sizeof(dir));
    rc = cloudsc_io_load_dir(dir, 1, &ds);
    if (!rc && o.reference_h5) {
      rc = cloudsc_io_load_hdf5_reference(o.reference_h5, &ds);     /* raw inputs, HDF5 reference */
      if (!rc) {
        size_t n = strlen(ds.source);
        snprintf(ds.source + n, sizeof(ds.source) - n, " + HDF5 %s (read-only)", o.reference_h5);
      }
    }
  }
  if (rc) {
    fprintf(stderr, "dwarf-cloudsc-amd: cannot load the input state: %s (%s)\n", cloudsc_strerror(rc),
            cloudsc_io_last_error());
    return EXIT_FAILURE;
  }
  if (o.write_h5_dir) {
    char a[PATH_MAX], b[PATH_MAX];
    snprintf(a, sizeof(a), "%s/input.h5", o.write_h5_dir);
    snprintf(b, sizeof(b), "%s/reference.h5", o.write_h5_dir);
    rc = cloudsc_io_write_hdf5(&ds, a, ds.has_reference ? b : NULL);
    if (rc) fprintf(stderr, "write failed: %s\n", cloudsc_io_last_error());
    else printf(" wrote %s%s%s\n", a, ds.has_reference ? " and " : "", ds.has_reference ? b : "");
    cloudsc_io_free(&ds);
    return rc ? EXIT_FAILURE : EXIT_SUCCESS;
  }

  if (o.variant == VARIANT_CPU) {
    if (o.precision != CLOUDSC_FP64 || o.ngpus != 1 || o.transfer) {
      fprintf(stderr, "dwarf-cloudsc-amd: --variant cpu runs fp64 on the host (no --gpus/--transfer/fp32)\n");
      cloudsc_io_free(&ds);
      return EXIT_FAILURE;
    }
    printf(" CLOUDSC-AMD: fp64, variant cpu (cloudsc_cpu_run, %d host thread(s)); state: %s\n", o.numomp,
           ds.source);
    if (o.energy_s > 0.0) printf(" ENERGY: n/a (host variant: no GPU board power)\n");
    rc = run_host(&o, &ds);
    cloudsc_io_free(&ds);
    return rc;
  }

  int ndev = 0;
  if ((rc = cloudsc_gpu_device_count(&ndev)) || ndev <= 0) {
    fprintf(stderr, "dwarf-cloudsc-amd: no HIP device (%s)\n", rc ? cloudsc_strerror(rc) : "0 devices");
    cloudsc_io_free(&ds);
    return EXIT_FAILURE;
  }
  if (o.ngpus > ndev)
    printf(" CLOUDSC-AMD: %d shards on %d visible device(s): shard d runs on device d %% %d\n", o.ngpus, ndev, ndev);

  if (o.transfer) {
    printf(" CLOUDSC-AMD: %s, variant %s, host-buffer path (--transfer), 1 device; state: %s\n",
           o.precision == CLOUDSC_FP64 ? "fp64" : "fp32",
           variant_name(o.variant),
           ds.source);
    if (o.energy_s > 0.0) printf(" ENERGY: n/a (the host-buffer path is bound by PCIe; run without --transfer)\n");
    rc = run_host(&o, &ds);
    cloudsc_io_free(&ds);
    return rc;
  }

  cloudsc_template_t tmpl;
  cloudsc_reference_t ref;
  cloudsc_io_template(&ds, &tmpl);
  cloudsc_io_reference(&ds, &ref);
  const int nblocks = o.ngptot / o.nproma + (o.ngptot % o.nproma ? 1 : 0);
  printf(" CLOUDSC-AMD: %s, variant %s, %d device(s); state: %s (KLON=%d, KLEV=%d)\n",
         o.precision == CLOUDSC_FP64 ? "fp64" : (o.exact_libm ? "fp32 (glibc expf/powf)" : "fp32"),
         variant_name(o.variant),
         o.ngpus, ds.source, ds.klon, ds.klev);

  /* the placement search costs ~0.5 s of kernel launches per state and saves
   * up to ~15 % per step: worth it for repeated steps, not for one (the
   * reference times a single launch, cloudsc_driver.cu:389-422) */
  const int place = o.place >= 0 ? o.place : o.reps > 1;
  cloudsc_set_placement_search(place ? -1 : 0);

  /* ---- shard: block-aligned contiguous ranges of the global column index ---- */
  shard_t *sh = (shard_t *)calloc((size_t)o.ngpus, sizeof(shard_t));
  pthread_t *th = (pthread_t *)calloc((size_t)o.ngpus, sizeof(pthread_t));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)o.ngpus);
  const int blocks_per = nblocks / o.ngpus, extra = nblocks % o.ngpus;
  long long col = 0;
  int nused = 0;
  for (int d = 0; d < o.ngpus; d++) {
    const int nb = blocks_per + (d < extra ? 1 : 0);
    long long cols = (long long)nb * o.nproma;
    if (col + cols > o.ngptot) cols = o.ngptot - col;
    if (cols <= 0) break;
    shard_t *s = &sh[nused++];
    s->device = d % ndev; s->ngptot = (int)cols; s->col_offset = col; s->nproma = o.nproma;
    s->precision = o.precision; s->variant = o.variant; s->reps = o.reps; s->warmup = o.warmup;
    s->libm_bit = o.exact_libm ? CLOUDSC_FP32_EXACT_LIBM : 0;
    s->energy_s = o.energy_s;
    s->tmpl = &tmpl; s->params = &ds.params; s->ref = ds.has_reference ? &ref : NULL; s->barrier = &bar;
    s->kernel_ms = (float *)calloc((size_t)o.reps, sizeof(float));
    col += cols;
  }
  if (nused != o.ngpus) {
    pthread_barrier_destroy(&bar);
    pthread_barrier_init(&bar, NULL, (unsigned)nused);
  }
  for (int d = 0; d < nused; d++) pthread_create(&th[d], NULL, shard_main, &sh[d]);
  for (int d = 0; d < nused; d++) pthread_join(th[d], NULL);
  pthread_barrier_destroy(&bar);

  int failed = 0;
  for (int d = 0; d < nused; d++)
    if (sh[d].rc) {
      fprintf(stderr, "dwarf-cloudsc-amd: shard %d (device %d): %s (%s)\n", d, sh[d].device,
              cloudsc_strerror(sh[d].rc), sh[d].err);
      failed = 1;
    }
  if (failed) { cloudsc_io_free(&ds); return EXIT_FAILURE; }

  /* ---- timing table (cloudsc_driver.c:233-262) ---- */
  double t0 = sh[0].t_start, t1 = sh[0].t_end;
  for (int d = 1; d < nused; d++) {
    if (sh[d].t_start < t0) t0 = sh[d].t_start;
    if (sh[d].t_end > t1) t1 = sh[d].t_end;
  }
  const double tdiff = t1 - t0;
  const double cols_done = (double)o.ngptot * o.reps;
  printf("     NUMOMP=%d, NGPTOT=%d, NPROMA=%d, NGPBLKS=%d\n", o.numomp, o.ngptot, o.nproma, nblocks);
  printf(" Reference MFLOP count for 100 columns : %12.8f\n", 1.0e-06 * ZHPM);
  printf(" %10s%10s%10s%10s%10s %4s : %10s%10s%10s\n", "NUMOMP", "NGPTOT", "#GP-cols", "#BLKS", "NPROMA", "tid#",
         "Time(msec)", "MFlops/s", "col/s");
  /* one row per shard, as the reference GPU driver prints one per host thread
   * (cloudsc_driver.cu:462-477): tid# = the shard (its host thread), and the row
   * ends in "@ core#" exactly as there, so JUBE's thr_time/thr_mflops patterns
   * (benchmark/include/include_patternset.yml:161-162) match it */
  for (int d = 0; d < nused; d++) {
    const double tl = sh[d].t_end - sh[d].t_start;
    const int nbd = sh[d].ngptot / o.nproma + (sh[d].ngptot % o.nproma ? 1 : 0);
    const double c = (double)sh[d].ngptot * o.reps;
    printf(" %10d%10d%10d%10d%10d %4d : %10d%10d%10d @ core#\n", o.numomp, o.ngptot, sh[d].ngptot, nbd, o.nproma,
           d, (int)(tl * 1000.), tl > 0 ? (int)(1.0e-06 * ZHPM * (c / 100.) / tl) : 0,
           tl > 0 ? (int)(c / tl) : 0);
  }
  printf(" %10d%10d%10d%10d%10d %4d : %10d%10d%10d TOTAL\n", o.numomp, o.ngptot, o.ngptot, nblocks, o.nproma, -1,
         (int)(tdiff * 1000.), tdiff > 0 ? (int)(1.0e-06 * ZHPM * (cols_done / 100.) / tdiff) : 0,
         tdiff > 0 ? (int)(cols_done / tdiff) : 0);
  /* precise figures for scripts (the table above keeps the reference's integer format) */
  double kmax = 0.0;
  for (int d = 0; d < nused; d++) {
    double k = 0.0;
    for (int r = 0; r < o.reps; r++) k += sh[d].kernel_ms[r];
    k /= o.reps;
    if (k > kmax) kmax = k;
  }
  printf(" TIMING: steps=%d wall_ms_per_step=%.4f kernel_ms_per_step=%.4f columns_per_s=%.1f devices=%d\n", o.reps,
         1e3 * tdiff / o.reps, kmax, cols_done / tdiff, nused);
  /* the placement search of each shard's state (cloudsc_state_placement_report) */
  for (int d = 0; d < nused; d++) {
    const cloudsc_placement_t *pl = &sh[d].place;
    if (pl->method == CLOUDSC_PLACE_METHOD_NONE) {
      printf(" PLACEMENT: shard=%d search=off\n", d);
      continue;
    }
    printf(" PLACEMENT: shard=%d search=kernel first_ms=%.4f kept_ms=%.4f tries=%d moves=%d launches=%d "
           "search_ms=%.1f peak_transient_MB=%.1f\n", d, pl->probe_first_ms, pl->probe_final_ms, pl->tries,
           pl->moves, pl->launches, pl->search_ms, pl->peak_transient_bytes / 1048576.0);
  }
  /* board power over the energy window (--energy): uJ per column = W x ms per launch / columns */
  for (int d = 0; d < nused && o.energy_s > 0.0; d++) {
    if (!sh[d].power_path[0] || !sh[d].power_samples) {
      printf(" ENERGY: shard=%d device=%d n/a (no hwmon power file for this device)\n", d, sh[d].device);
      continue;
    }
    /* shards sharing a device (--gpus above the device count) read the same
     * board over overlapping windows: the board's power is not theirs alone
     * (ADVICE r05), so no per-column figure is claimed */
    int sharing = 0;
    for (int e = 0; e < nused; e++) sharing += sh[e].device == sh[d].device;
    if (sharing > 1) {
      printf(" ENERGY: shard=%d device=%d board_w=%.1f samples=%d uj_per_column=n/a (the device runs %d shards "
             "at once; its board power is theirs together)\n", d, sh[d].device, sh[d].board_w,
             sh[d].power_samples, sharing);
      continue;
    }
    printf(" ENERGY: shard=%d device=%d board_w=%.1f samples=%d steps=%d ms_per_step=%.4f uj_per_column=%.3f "
           "source=%s\n", d, sh[d].device, sh[d].board_w, sh[d].power_samples, sh[d].energy_steps,
           sh[d].energy_ms_per_step, sh[d].board_w * sh[d].energy_ms_per_step * 1e3 / sh[d].ngptot,
           sh[d].power_path);
  }

  /* ---- validation (cloudsc_validate.c:193-216, combined over devices) ---- */
  int bad = 0;
  if (ds.has_reference) {
    printf(" %20s %s %20s %20s %20s %20s %20s\n", "Variable", "Dim", "MinValue", "MaxValue", "AbsMaxErr",
           "AvgAbsErr/GP", "MaxRelErr-%");
    const int gate = o.precision == CLOUDSC_FP64 || o.tol_given;
    double worst = 0.0;
    for (int f = 0; f < CLOUDSC_NVALID; f++) {
      cloudsc_stats_t s = sh[0].stats[f];
      for (int d = 1; d < nused; d++) cloudsc_stats_combine(&s, &sh[d].stats[f]);   /* double-double sums */
      const int kind = cloudsc_io_ref_kind[f];
      const double rel = print_error(cloudsc_io_print_names[f], kind == 3 ? 1 : kind == 2 ? 3 : 2, &s, o.ngptot);
      if (rel > worst) worst = rel;
      if (gate && !(rel <= o.tol)) bad++;
    }
    if (gate)
      printf(" VALIDATION: %s (worst relative L1 error %.3e, gate %.1e, %d field(s) over)\n",
             bad ? "FAILED" : "PASSED", worst, o.tol, bad);
    else
      printf(" VALIDATION: reported only (fp32 vs the fp64 reference; worst relative L1 error %.3e)\n", worst);
  } else {
    printf(" VALIDATION: skipped (no reference outputs loaded)\n");
  }
  for (int d = 0; d < nused; d++) free(sh[d].kernel_ms);
  free(sh);
  free(th);
  cloudsc_io_free(&ds);
  return bad ? EXIT_FAILURE : EXIT_SUCCESS;
}
