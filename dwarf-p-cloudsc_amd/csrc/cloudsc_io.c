/*
 * cloudsc_io.c -- dataset plumbing of the dwarf host driver: raw and HDF5
 * readers (HDF5 through a dlopen'ed libhdf5, files opened read-only), the
 * input.h5 / reference.h5 writer, and views for the C ABI.  See cloudsc_io.h.
 *
 * Field and scalar names follow the reference's HDF5 reader
 * (src/cloudsc_c/cloudsc/load_state.c:499-690 inputs and parameters,
 * :746-800 reference outputs).
 */
#define _GNU_SOURCE
#include "cloudsc_io.h"

#include <ctype.h>
#include <float.h>
#include <math.h>
#include <dlfcn.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char g_err[512];
static void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char *cloudsc_io_last_error(void) { return g_err; }

const char *const cloudsc_io_input_names[CLOUDSC_IO_NIN] = {
    "PT", "PQ", "TENDENCY_TMP_T", "TENDENCY_TMP_Q", "TENDENCY_TMP_A", "TENDENCY_TMP_CLD",
    "PVFL", "PVFI", "PHRSW", "PHRLW", "PVERVEL", "PAP", "PAPH", "PLSM", "KTYPE",
    "PLU", "PLUDE", "PSNDE", "PMFU", "PMFD", "PA", "PCLV", "PSUPSAT",
    "PLCRIT_AER", "PICRIT_AER", "PRE_ICE", "PCCN", "PNICE"};
const int cloudsc_io_input_kind[CLOUDSC_IO_NIN] = {
    0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0, 1, 3, 3, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0};

const char *const cloudsc_io_ref_names[CLOUDSC_NVALID] = {
    "PLUDE", "PCOVPTOT", "PRAINFRAC_TOPRFZ", "PFSQLF", "PFSQIF", "PFCQLNG", "PFCQNNG",
    "PFSQRF", "PFSQSF", "PFCQRNG", "PFCQSNG", "PFSQLTUR", "PFSQITUR", "PFPLSL", "PFPLSN",
    "PFHPSL", "PFHPSN", "TENDENCY_LOC_A", "TENDENCY_LOC_Q", "TENDENCY_LOC_T", "TENDENCY_LOC_CLD"};
const char *const cloudsc_io_print_names[CLOUDSC_NVALID] = {
    "PLUDE", "PCOVPTOT", "PRAINFRAC_TOPRFZ", "PFSQLF", "PFSQIF", "PFCQLNG", "PFCQNNG",
    "PFSQRF", "PFSQSF", "PFCQRNG", "PFCQSNG", "PFSQLTUR", "PFSQITUR", "PFPLSL", "PFPLSN",
    "PFHPSL", "PFHPSN", "TENDENCY_LOC%A", "TENDENCY_LOC%Q", "TENDENCY_LOC%T", "TENDENCY_LOC%CLD"};
const int cloudsc_io_ref_kind[CLOUDSC_NVALID] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 2};

/* HDF5 scalar names, in cloudsc_params_t order (doubles ptsphy..nshapeq, then
 * the ints); the raw params.txt uses the same names lower-cased without the
 * YRECLDP_ prefix */
static const char *const k_param_double_names[] = {
    "PTSPHY", "RG", "RD", "RCPD", "RETV", "RLVTT", "RLSTT", "RLMLT", "RTT", "RV", "R2ES", "R3LES", "R3IES",
    "R4LES", "R4IES", "R5LES", "R5IES", "R5ALVCP", "R5ALSCP", "RALVDCP", "RALSDCP", "RALFDCP", "RTWAT",
    "RTICE", "RTICECU", "RTWAT_RTICE_R", "RTWAT_RTICECU_R", "RKOOP1", "RKOOP2", "YRECLDP_RAMID",
    "YRECLDP_RCLDIFF", "YRECLDP_RCLDIFF_CONVI", "YRECLDP_RCLCRIT", "YRECLDP_RCLCRIT_SEA",
    "YRECLDP_RCLCRIT_LAND", "YRECLDP_RKCONV", "YRECLDP_RPRC1", "YRECLDP_RPRC2", "YRECLDP_RCLDMAX",
    "YRECLDP_RPECONS", "YRECLDP_RVRFACTOR", "YRECLDP_RPRECRHMAX", "YRECLDP_RTAUMEL", "YRECLDP_RAMIN",
    "YRECLDP_RLMIN", "YRECLDP_RKOOPTAU", "YRECLDP_RCLDTOPP", "YRECLDP_RLCRITSNOW", "YRECLDP_RSNOWLIN1",
    "YRECLDP_RSNOWLIN2", "YRECLDP_RICEHI1", "YRECLDP_RICEHI2", "YRECLDP_RICEINIT", "YRECLDP_RVICE",
    "YRECLDP_RVRAIN", "YRECLDP_RVSNOW", "YRECLDP_RTHOMO", "YRECLDP_RCOVPMIN", "YRECLDP_RCCN", "YRECLDP_RNICE",
    "YRECLDP_RCCNOM", "YRECLDP_RCCNSS", "YRECLDP_RCCNSU", "YRECLDP_RCLDTOPCF", "YRECLDP_RDEPLIQREFRATE",
    "YRECLDP_RDEPLIQREFDEPTH", "YRECLDP_RCL_KKAac", "YRECLDP_RCL_KKBac", "YRECLDP_RCL_KKAau",
    "YRECLDP_RCL_KKBauq", "YRECLDP_RCL_KKBaun", "YRECLDP_RCL_KK_cloud_num_sea",
    "YRECLDP_RCL_KK_cloud_num_land", "YRECLDP_RCL_AI", "YRECLDP_RCL_BI", "YRECLDP_RCL_CI", "YRECLDP_RCL_DI",
    "YRECLDP_RCL_X1I", "YRECLDP_RCL_X2I", "YRECLDP_RCL_X3I", "YRECLDP_RCL_X4I", "YRECLDP_RCL_CONST1I",
    "YRECLDP_RCL_CONST2I", "YRECLDP_RCL_CONST3I", "YRECLDP_RCL_CONST4I", "YRECLDP_RCL_CONST5I",
    "YRECLDP_RCL_CONST6I", "YRECLDP_RCL_APB1", "YRECLDP_RCL_APB2", "YRECLDP_RCL_APB3", "YRECLDP_RCL_AS",
    "YRECLDP_RCL_BS", "YRECLDP_RCL_CS", "YRECLDP_RCL_DS", "YRECLDP_RCL_X1S", "YRECLDP_RCL_X2S",
    "YRECLDP_RCL_X3S", "YRECLDP_RCL_X4S", "YRECLDP_RCL_CONST1S", "YRECLDP_RCL_CONST2S", "YRECLDP_RCL_CONST3S",
    "YRECLDP_RCL_CONST4S", "YRECLDP_RCL_CONST5S", "YRECLDP_RCL_CONST6S", "YRECLDP_RCL_CONST7S",
    "YRECLDP_RCL_CONST8S", "YRECLDP_RDENSWAT", "YRECLDP_RDENSREF", "YRECLDP_RCL_AR", "YRECLDP_RCL_BR",
    "YRECLDP_RCL_CR", "YRECLDP_RCL_DR", "YRECLDP_RCL_X1R", "YRECLDP_RCL_X2R", "YRECLDP_RCL_X4R",
    "YRECLDP_RCL_KA273", "YRECLDP_RCL_CDENOM1", "YRECLDP_RCL_CDENOM2", "YRECLDP_RCL_CDENOM3",
    "YRECLDP_RCL_SCHMIDT", "YRECLDP_RCL_DYNVISC", "YRECLDP_RCL_CONST1R", "YRECLDP_RCL_CONST2R",
    "YRECLDP_RCL_CONST3R", "YRECLDP_RCL_CONST4R", "YRECLDP_RCL_FAC1", "YRECLDP_RCL_FAC2",
    "YRECLDP_RCL_CONST5R", "YRECLDP_RCL_CONST6R", "YRECLDP_RCL_FZRAB", "YRECLDP_RCL_FZRBB", "YRECLDP_NSHAPEP",
    "YRECLDP_NSHAPEQ",
};
static const char *const k_param_int_names[] = {
    "YRECLDP_LCLDEXTRA", "YRECLDP_LCLDBUDGET", "YRECLDP_NSSOPT", "YRECLDP_NCLDTOP", "YRECLDP_NAECLBC",
    "YRECLDP_NAECLDU", "YRECLDP_NAECLOM", "YRECLDP_NAECLSS", "YRECLDP_NAECLSU", "YRECLDP_NCLDDIAG",
    "YRECLDP_NAERCLD", "YRECLDP_LAERLIQAUTOLSP", "YRECLDP_LAERLIQAUTOCP", "YRECLDP_LAERLIQAUTOCPB",
    "YRECLDP_LAERLIQCOLL", "YRECLDP_LAERICESED", "YRECLDP_LAERICEAUTO", "YRECLDP_NBETA",
};
#define N_PDOUBLE ((int)(sizeof(k_param_double_names) / sizeof(k_param_double_names[0])))
#define N_PINT ((int)(sizeof(k_param_int_names) / sizeof(k_param_int_names[0])))

static double *param_doubles(cloudsc_params_t *p) { return &p->ptsphy; }
static int *param_ints(cloudsc_params_t *p) { return &p->lcldextra; }
static const double *cparam_doubles(const cloudsc_params_t *p) { return &p->ptsphy; }
static const int *cparam_ints(const cloudsc_params_t *p) { return &p->lcldextra; }

/* params.txt key of an HDF5 scalar name */
static void raw_key(const char *h5name, char *out, size_t n) {
  const char *s = strncmp(h5name, "YRECLDP_", 8) == 0 ? h5name + 8 : h5name;
  size_t i = 0;
  for (; s[i] && i + 1 < n; i++) out[i] = (char)tolower((unsigned char)s[i]);
  out[i] = 0;
}

long long cloudsc_io_elems(int kind, int klev, int klon) {
  switch (kind) {
    case 0: return (long long)klev * klon;
    case 1: return (long long)(klev + 1) * klon;
    case 2: return (long long)CLOUDSC_NCLV * klev * klon;
    default: return klon;
  }
}

void cloudsc_io_free(cloudsc_dataset_t *ds) {
  if (!ds) return;
  for (int i = 0; i < CLOUDSC_IO_NIN; i++) free(ds->in[i]);
  free(ds->ktype);
  for (int i = 0; i < CLOUDSC_NVALID; i++) free(ds->ref[i]);
  memset(ds, 0, sizeof(*ds));
}

static int check_layout(void) {
  /* the parameter block is read as one run of doubles and one run of ints */
  cloudsc_params_t p;
  if ((char *)&p.nshapeq - (char *)&p.ptsphy != (long)sizeof(double) * (N_PDOUBLE - 1)) return 0;
  if ((char *)&p.nbeta - (char *)&p.lcldextra != (long)sizeof(int) * (N_PINT - 1)) return 0;
  return 1;
}

/* ------------------------------------------------------------------------ */
/* raw directory                                                             */
/* ------------------------------------------------------------------------ */
static void *read_file(const char *path, size_t expect_bytes, int *rc) {
  FILE *f = fopen(path, "rb");
  if (!f) { *rc = CLOUDSC_EIO; set_err("cannot open %s", path); return NULL; }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (sz < 0 || (size_t)sz != expect_bytes) {
    fclose(f);
    *rc = CLOUDSC_EIO;
    set_err("%s: %ld bytes, expected %zu", path, sz, expect_bytes);
    return NULL;
  }
  void *buf = malloc(expect_bytes ? expect_bytes : 1);
  if (!buf) { fclose(f); *rc = CLOUDSC_ENOMEM; return NULL; }
  if (fread(buf, 1, expect_bytes, f) != expect_bytes) {
    free(buf); fclose(f); *rc = CLOUDSC_EIO; set_err("short read on %s", path); return NULL;
  }
  fclose(f);
  *rc = CLOUDSC_OK;
  return buf;
}

static int file_exists(const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return 0;
  fclose(f);
  return 1;
}

/* "klon": N in manifest.json (a flat JSON object) */
static int json_int(const char *text, const char *key, int *out) {
  char pat[64];
  snprintf(pat, sizeof(pat), "\"%s\"", key);
  const char *p = strstr(text, pat);
  if (!p) return 0;
  p = strchr(p + strlen(pat), ':');
  if (!p) return 0;
  *out = atoi(p + 1);
  return 1;
}

static int load_params_txt(const char *path, cloudsc_params_t *p) {
  FILE *f = fopen(path, "r");
  if (!f) { set_err("cannot open %s", path); return CLOUDSC_EIO; }
  unsigned char seen_d[256] = {0}, seen_i[64] = {0};
  char line[512];
  while (fgets(line, sizeof(line), f)) {
    char *h = strchr(line, '#');
    if (h) *h = 0;
    char *eq = strchr(line, '=');
    if (!eq) continue;
    *eq = 0;
    char name[128];
    if (sscanf(line, " %127s", name) != 1) continue;
    const char *val = eq + 1;
    char key[128];
    int found = 0;
    for (int i = 0; i < N_PDOUBLE && !found; i++) {
      raw_key(k_param_double_names[i], key, sizeof(key));
      if (!strcmp(key, name)) { param_doubles(p)[i] = strtod(val, NULL); seen_d[i] = 1; found = 1; }
    }
    for (int i = 0; i < N_PINT && !found; i++) {
      raw_key(k_param_int_names[i], key, sizeof(key));
      if (!strcmp(key, name)) { param_ints(p)[i] = (int)strtol(val, NULL, 10); seen_i[i] = 1; found = 1; }
    }
  }
  fclose(f);
  for (int i = 0; i < N_PDOUBLE; i++)
    if (!seen_d[i]) { set_err("%s: missing %s", path, k_param_double_names[i]); return CLOUDSC_EIO; }
  for (int i = 0; i < N_PINT; i++)
    if (!seen_i[i]) { set_err("%s: missing %s", path, k_param_int_names[i]); return CLOUDSC_EIO; }
  return CLOUDSC_OK;
}

/* ------------------------------------------------------------------------ */
/* Serialbox store (the reference's data/ directory): MetaData-<prefix>.json  */
/* (global_meta_info: KLON, KLEV and the parameter scalars under the same     */
/* names as input.h5; field_map: dims and element type of every field),       */
/* ArchiveMetaData-<prefix>.json (fields_table: byte offset of each field in  */
/* <prefix>_<FIELD>.dat per savepoint), the .dat files raw column-major       */
/* (Fortran) arrays -- i.e. C-order [..][lev][klon].  This is what            */
/* serialbox2hdf5/serialbox2hdf5.py:11-33 converts into input.h5, read here    */
/* directly (the scalars the way load_state.c:538-690 reads them from HDF5).  */
/* ------------------------------------------------------------------------ */
typedef struct jv {
  int type;                         /* 0 null, 1 bool, 2 number, 3 string, 4 array, 5 object */
  double num;
  char *str;
  int n;
  struct jv *items;                 /* array elements / object values */
  char **keys;                      /* object keys */
} jv;

static void jv_free(jv *v) {
  if (!v) return;
  free(v->str);
  for (int i = 0; i < v->n; i++) {
    jv_free(&v->items[i]);
    if (v->keys) free(v->keys[i]);
  }
  free(v->items);
  free(v->keys);
  memset(v, 0, sizeof(*v));
}

typedef struct { const char *p, *end; int err; } jparser;

static void jws(jparser *j) {
  while (j->p < j->end && (*j->p == ' ' || *j->p == '\n' || *j->p == '\r' || *j->p == '\t')) j->p++;
}
static char *jstring(jparser *j) {
  if (j->p >= j->end || *j->p != '"') { j->err = 1; return NULL; }
  j->p++;
  size_t cap = 16, n = 0;
  char *out = (char *)malloc(cap);
  while (out && j->p < j->end && *j->p != '"') {
    char c = *j->p++;
    if (c == '\\' && j->p < j->end) {
      c = *j->p++;
      if (c == 'n') c = '\n'; else if (c == 't') c = '\t'; else if (c == 'u') { j->p += 4; c = '?'; }
    }
    if (n + 2 > cap) { cap *= 2; char *t = (char *)realloc(out, cap); if (!t) { free(out); out = NULL; break; } out = t; }
    out[n++] = c;
  }
  if (!out || j->p >= j->end) { free(out); j->err = 1; return NULL; }
  j->p++;
  out[n] = 0;
  return out;
}
static int jvalue(jparser *j, jv *v, int depth) {
  memset(v, 0, sizeof(*v));
  jws(j);
  if (j->p >= j->end || depth > 64) return j->err = 1;
  const char c = *j->p;
  if (c == '{' || c == '[') {
    const int obj = c == '{';
    v->type = obj ? 5 : 4;
    j->p++;
    int cap = 0;
    for (;;) {
      jws(j);
      if (j->p < j->end && *j->p == (obj ? '}' : ']')) { j->p++; return 0; }
      if (v->n == cap) {
        cap = cap ? 2 * cap : 8;
        jv *ni = (jv *)realloc(v->items, sizeof(jv) * cap);
        if (!ni) return j->err = 1;
        v->items = ni;
        if (obj) {
          char **nk = (char **)realloc(v->keys, sizeof(char *) * cap);
          if (!nk) return j->err = 1;
          v->keys = nk;
        }
      }
      if (obj) {
        v->keys[v->n] = NULL;
        memset(&v->items[v->n], 0, sizeof(jv));
        char *k = jstring(j);
        if (!k) return j->err = 1;
        v->keys[v->n] = k;
        jws(j);
        if (j->p >= j->end || *j->p != ':') { v->n++; return j->err = 1; }
        j->p++;
      }
      const int r = jvalue(j, &v->items[v->n], depth + 1);
      v->n++;
      if (r) return j->err = 1;
      jws(j);
      if (j->p < j->end && *j->p == ',') { j->p++; continue; }
      if (j->p < j->end && *j->p == (obj ? '}' : ']')) { j->p++; return 0; }
      return j->err = 1;
    }
  }
  if (c == '"') { v->type = 3; v->str = jstring(j); return v->str ? 0 : (j->err = 1); }
  /* the text is not NUL-terminated: every look-ahead is bounded by j->end */
  const size_t left = (size_t)(j->end - j->p);
  if (left >= 4 && !memcmp(j->p, "true", 4)) { v->type = 1; v->num = 1; j->p += 4; return 0; }
  if (left >= 5 && !memcmp(j->p, "false", 5)) { v->type = 1; v->num = 0; j->p += 5; return 0; }
  if (left >= 4 && !memcmp(j->p, "null", 4)) { v->type = 0; j->p += 4; return 0; }
  /* a number: its characters copied into a NUL-terminated buffer first, so
   * strtod cannot read past the end of a file truncated inside the number */
  char num[64];
  size_t n = 0;
  while (n < left && n < sizeof(num) - 1 && strchr("+-0123456789.eE", j->p[n]) && j->p[n]) n++;
  if (n == 0 || n == sizeof(num) - 1) return j->err = 1;
  memcpy(num, j->p, n);
  num[n] = 0;
  char *e = NULL;
  v->num = strtod(num, &e);      /* decimal -> double, correctly rounded by the C library */
  if (e == num) return j->err = 1;
  v->type = 2;
  j->p += e - num;
  return 0;
}
static const jv *jget(const jv *o, const char *key) {
  if (!o || o->type != 5) return NULL;
  for (int i = 0; i < o->n; i++)
    if (!strcmp(o->keys[i], key)) return &o->items[i];
  return NULL;
}
static int jparse_file(const char *path, jv *root) {
  memset(root, 0, sizeof(*root));
  FILE *f = fopen(path, "rb");
  if (!f) { set_err("cannot open %s", path); return CLOUDSC_EIO; }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *text = sz > 0 ? (char *)malloc((size_t)sz) : NULL;
  if (!text || fread(text, 1, (size_t)sz, f) != (size_t)sz) {
    free(text); fclose(f); set_err("cannot read %s", path); return CLOUDSC_EIO;
  }
  fclose(f);
  jparser j = {text, text + sz, 0};
  jvalue(&j, root, 0);
  free(text);
  if (j.err || root->type != 5) { jv_free(root); set_err("%s: not a JSON object", path); return CLOUDSC_EIO; }
  return CLOUDSC_OK;
}

/* one Serialbox field: checks dims / element type, reads it at its archive offset */
static void *sb_read_field(const char *dir, const char *prefix, const jv *meta, const jv *archive,
                           const char *name, long long expect, int want_int, int *rc) {
  const jv *fm = jget(jget(meta, "field_map"), name);
  if (!fm) { *rc = CLOUDSC_EIO; set_err("Serialbox %s: no field %s", prefix, name); return NULL; }
  const jv *dims = jget(fm, "dims");
  long long ne = 1;
  for (int i = 0; dims && dims->type == 4 && i < dims->n; i++) ne *= (long long)dims->items[i].num;
  const jv *mi = jget(fm, "meta_info");
  const jv *et = jget(jget(mi, "__elementtype"), "value");
  const jv *bpe = jget(jget(mi, "__bytesperelement"), "value");
  const int esz = bpe ? (int)bpe->num : 0;
  const int is_int = et && et->str && !strcmp(et->str, "int");
  const int is_dbl = et && et->str && !strcmp(et->str, "double");
  if (ne != expect || (want_int ? !(is_int && esz == 4) : !(is_dbl && esz == 8))) {
    *rc = CLOUDSC_EIO;
    set_err("Serialbox %s: field %s has %lld elements of %s/%d B, expected %lld of %s", prefix, name, ne,
            et && et->str ? et->str : "?", esz, expect, want_int ? "int32" : "double");
    return NULL;
  }
  long long offset = 0;
  const jv *ft = jget(jget(archive, "fields_table"), name);   /* [[offset, checksum], ...] per savepoint */
  if (ft && ft->type == 4 && ft->n > 0 && ft->items[0].type == 4 && ft->items[0].n > 0)
    offset = (long long)ft->items[0].items[0].num;
  char path[1024];
  snprintf(path, sizeof(path), "%s/%s_%s.dat", dir, prefix, name);
  FILE *f = fopen(path, "rb");
  if (!f) { *rc = CLOUDSC_EIO; set_err("cannot open %s", path); return NULL; }
  const size_t bytes = (size_t)ne * (size_t)esz;
  void *buf = malloc(bytes ? bytes : 1);
  if (!buf || fseek(f, (long)offset, SEEK_SET) != 0 || fread(buf, 1, bytes, f) != bytes) {
    free(buf); fclose(f); *rc = buf ? CLOUDSC_EIO : CLOUDSC_ENOMEM; set_err("short read on %s", path); return NULL;
  }
  fclose(f);
  *rc = CLOUDSC_OK;
  return buf;
}

int cloudsc_io_load_serialbox(const char *dir, int with_reference, cloudsc_dataset_t *ds) {
  if (!dir || !ds) return CLOUDSC_EINVAL;
  if (!check_layout()) { set_err("cloudsc_params_t layout mismatch"); return CLOUDSC_EINVAL; }
  memset(ds, 0, sizeof(*ds));
  char path[1024];
  jv meta, arch;
  int rc;
  snprintf(path, sizeof(path), "%s/MetaData-input.json", dir);
  if ((rc = jparse_file(path, &meta))) return rc;
  snprintf(path, sizeof(path), "%s/ArchiveMetaData-input.json", dir);
  if ((rc = jparse_file(path, &arch))) { jv_free(&meta); return rc; }
  const jv *g = jget(&meta, "global_meta_info");
  const jv *klon = jget(jget(g, "KLON"), "value"), *klev = jget(jget(g, "KLEV"), "value");
  rc = CLOUDSC_OK;
  if (!klon || !klev || klon->num <= 0 || klev->num < 2) { set_err("%s: no KLON/KLEV", dir); rc = CLOUDSC_EIO; }
  if (!rc) { ds->klon = (int)klon->num; ds->klev = (int)klev->num; }
  /* parameters: the input.h5 scalar names (logicals -> 0/1, like hdf5_file_mod.F90:171-175) */
  for (int i = 0; i < N_PDOUBLE && !rc; i++) {
    const jv *v = jget(jget(g, k_param_double_names[i]), "value");
    if (!v || (v->type != 2 && v->type != 1)) { set_err("%s: missing scalar %s", dir, k_param_double_names[i]); rc = CLOUDSC_EIO; }
    else param_doubles(&ds->params)[i] = v->num;
  }
  for (int i = 0; i < N_PINT && !rc; i++) {
    const jv *v = jget(jget(g, k_param_int_names[i]), "value");
    if (!v || (v->type != 2 && v->type != 1)) { set_err("%s: missing scalar %s", dir, k_param_int_names[i]); rc = CLOUDSC_EIO; }
    else param_ints(&ds->params)[i] = (int)v->num;
  }
  for (int i = 0; i < CLOUDSC_IO_NIN && !rc; i++) {
    const char *name = cloudsc_io_input_names[i];
    if (i >= CLOUDSC_IO_FIRST_AEROSOL) {          /* aerosol inputs are optional (read only under LAER*) */
      snprintf(path, sizeof(path), "%s/input_%s.dat", dir, name);
      if (!jget(jget(&meta, "field_map"), name) || !file_exists(path)) continue;
    }
    const long long ne = cloudsc_io_elems(cloudsc_io_input_kind[i], ds->klev, ds->klon);
    void *buf = sb_read_field(dir, "input", &meta, &arch, name, ne, i == CLOUDSC_IO_KTYPE, &rc);
    if (i == CLOUDSC_IO_KTYPE) ds->ktype = (int *)buf;
    else ds->in[i] = (double *)buf;
  }
  jv_free(&meta);
  jv_free(&arch);
  if (!rc && with_reference) {
    snprintf(path, sizeof(path), "%s/MetaData-reference.json", dir);
    if (!(rc = jparse_file(path, &meta))) {
      snprintf(path, sizeof(path), "%s/ArchiveMetaData-reference.json", dir);
      if (!(rc = jparse_file(path, &arch))) {
        for (int i = 0; i < CLOUDSC_NVALID && !rc; i++) {
          const long long ne = cloudsc_io_elems(cloudsc_io_ref_kind[i], ds->klev, ds->klon);
          ds->ref[i] = (double *)sb_read_field(dir, "reference", &meta, &arch, cloudsc_io_ref_names[i], ne, 0, &rc);
        }
        jv_free(&arch);
      }
      jv_free(&meta);
    }
    if (!rc) ds->has_reference = 1;
  }
  if (rc) { cloudsc_io_free(ds); return rc; }
  snprintf(ds->source, sizeof(ds->source), "Serialbox store %s", dir);
  return CLOUDSC_OK;
}

int cloudsc_io_load_raw(const char *dir, int with_reference, cloudsc_dataset_t *ds) {
  if (!dir || !ds) return CLOUDSC_EINVAL;
  if (!check_layout()) { set_err("cloudsc_params_t layout mismatch"); return CLOUDSC_EINVAL; }
  memset(ds, 0, sizeof(*ds));
  char path[1024];
  int rc;
  snprintf(path, sizeof(path), "%s/manifest.json", dir);
  FILE *f = fopen(path, "r");
  if (!f) { set_err("cannot open %s", path); return CLOUDSC_EIO; }
  char text[8192];
  size_t n = fread(text, 1, sizeof(text) - 1, f);
  fclose(f);
  text[n] = 0;
  if (!json_int(text, "klon", &ds->klon) || !json_int(text, "klev", &ds->klev) || ds->klon <= 0 ||
      ds->klev < 2) {
    set_err("%s: no klon/klev", path);
    return CLOUDSC_EIO;
  }
  snprintf(path, sizeof(path), "%s/params.txt", dir);
  if ((rc = load_params_txt(path, &ds->params))) { cloudsc_io_free(ds); return rc; }
  for (int i = 0; i < CLOUDSC_IO_NIN; i++) {
    snprintf(path, sizeof(path), "%s/input_%s.dat", dir, cloudsc_io_input_names[i]);
    const long long ne = cloudsc_io_elems(cloudsc_io_input_kind[i], ds->klev, ds->klon);
    if (i >= CLOUDSC_IO_FIRST_AEROSOL && !file_exists(path)) continue;    /* optional */
    if (i == CLOUDSC_IO_KTYPE) {
      ds->ktype = (int *)read_file(path, (size_t)ne * sizeof(int), &rc);
      if (!ds->ktype) { cloudsc_io_free(ds); return rc; }
    } else {
      ds->in[i] = (double *)read_file(path, (size_t)ne * sizeof(double), &rc);
      if (!ds->in[i]) { cloudsc_io_free(ds); return rc; }
    }
  }
  if (with_reference) {
    for (int i = 0; i < CLOUDSC_NVALID; i++) {
      snprintf(path, sizeof(path), "%s/reference_%s.dat", dir, cloudsc_io_ref_names[i]);
      const long long ne = cloudsc_io_elems(cloudsc_io_ref_kind[i], ds->klev, ds->klon);
      ds->ref[i] = (double *)read_file(path, (size_t)ne * sizeof(double), &rc);
      if (!ds->ref[i]) { cloudsc_io_free(ds); return rc; }
    }
    ds->has_reference = 1;
  }
  snprintf(ds->source, sizeof(ds->source), "raw dataset %s", dir);
  return CLOUDSC_OK;
}

/* ------------------------------------------------------------------------ */
/* HDF5 through dlopen (HDF5 >= 1.10: hid_t is 64-bit)                       */
/* ------------------------------------------------------------------------ */
typedef int64_t hid_t;
typedef int herr_t;
typedef unsigned long long hsize_t;
#define H5P_DEFAULT_ ((hid_t)0)
#define H5S_ALL_ ((hid_t)0)
#define H5E_DEFAULT_ ((hid_t)0)
#define H5F_ACC_RDONLY_ 0x0000u
#define H5F_ACC_TRUNC_ 0x0002u

static struct {
  int tried, ok;
  void *h;
  herr_t (*open)(void);
  herr_t (*get_libversion)(unsigned *, unsigned *, unsigned *);
  herr_t (*eset_auto2)(hid_t, void *, void *);
  hid_t (*fopen)(const char *, unsigned, hid_t);
  hid_t (*fcreate)(const char *, unsigned, hid_t, hid_t);
  herr_t (*fclose)(hid_t);
  hid_t (*dopen2)(hid_t, const char *, hid_t);
  hid_t (*dcreate2)(hid_t, const char *, hid_t, hid_t, hid_t, hid_t, hid_t);
  herr_t (*dread)(hid_t, hid_t, hid_t, hid_t, hid_t, void *);
  herr_t (*dwrite)(hid_t, hid_t, hid_t, hid_t, hid_t, const void *);
  hid_t (*dget_space)(hid_t);
  herr_t (*dclose)(hid_t);
  int (*s_ndims)(hid_t);
  int (*s_dims)(hid_t, hsize_t *, hsize_t *);
  hid_t (*s_create_simple)(int, const hsize_t *, const hsize_t *);
  herr_t (*sclose)(hid_t);
  hid_t *native_double, *native_int, *ieee_f64le, *std_i32le, *std_i64le, *native_llong;
} H5;

static int h5_load(void) {
  if (H5.tried) return H5.ok;
  H5.tried = 1;
  const char *cands[] = {getenv("CLOUDSC_HDF5_LIB"), "libhdf5.so", "libhdf5.so.103", "libhdf5.so.200",
                         "/opt/conda/lib/libhdf5.so", "/opt/conda/lib/libhdf5.so.103",
                         "/usr/lib/x86_64-linux-gnu/hdf5/serial/libhdf5.so"};
  for (size_t i = 0; i < sizeof(cands) / sizeof(cands[0]) && !H5.h; i++)
    if (cands[i] && *cands[i]) H5.h = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
  if (!H5.h) { set_err("libhdf5 not found (set CLOUDSC_HDF5_LIB)"); return 0; }
#define SYM(field, name)                                               \
  do {                                                                 \
    *(void **)(&H5.field) = dlsym(H5.h, name);                         \
    if (!H5.field) { set_err("libhdf5: no symbol %s", name); return 0; } \
  } while (0)
  SYM(open, "H5open"); SYM(get_libversion, "H5get_libversion"); SYM(eset_auto2, "H5Eset_auto2");
  SYM(fopen, "H5Fopen"); SYM(fcreate, "H5Fcreate"); SYM(fclose, "H5Fclose");
  SYM(dopen2, "H5Dopen2"); SYM(dcreate2, "H5Dcreate2"); SYM(dread, "H5Dread"); SYM(dwrite, "H5Dwrite");
  SYM(dget_space, "H5Dget_space"); SYM(dclose, "H5Dclose");
  SYM(s_ndims, "H5Sget_simple_extent_ndims"); SYM(s_dims, "H5Sget_simple_extent_dims");
  SYM(s_create_simple, "H5Screate_simple"); SYM(sclose, "H5Sclose");
  SYM(native_double, "H5T_NATIVE_DOUBLE_g"); SYM(native_int, "H5T_NATIVE_INT_g");
  SYM(native_llong, "H5T_NATIVE_LLONG_g"); SYM(ieee_f64le, "H5T_IEEE_F64LE_g");
  SYM(std_i32le, "H5T_STD_I32LE_g"); SYM(std_i64le, "H5T_STD_I64LE_g");
#undef SYM
  if (H5.open() < 0) { set_err("H5open failed"); return 0; }
  unsigned maj = 0, min = 0, rel = 0;
  H5.get_libversion(&maj, &min, &rel);
  if (maj < 1 || (maj == 1 && min < 10)) { set_err("libhdf5 %u.%u too old (need >= 1.10)", maj, min); return 0; }
  H5.eset_auto2(H5E_DEFAULT_, NULL, NULL);     /* errors are reported by return codes */
  H5.ok = 1;
  return 1;
}

int cloudsc_io_hdf5_available(void) { return h5_load(); }

/* read a whole dataset of `expect` elements (any rank) as double or int */
static int h5_read(hid_t file, const char *name, long long expect, int as_int, void *buf) {
  char path[160];
  snprintf(path, sizeof(path), "/%s", name);
  hid_t d = H5.dopen2(file, path, H5P_DEFAULT_);
  if (d < 0) { set_err("HDF5 dataset %s not found", path); return CLOUDSC_EIO; }
  hid_t s = H5.dget_space(d);
  int nd = s >= 0 ? H5.s_ndims(s) : -1;
  hsize_t dims[8];
  long long n = 1;
  if (nd < 0 || nd > 8 || H5.s_dims(s, dims, NULL) < 0) n = -1;
  else for (int i = 0; i < nd; i++) n *= (long long)dims[i];
  if (s >= 0) H5.sclose(s);
  if (n != expect) {
    H5.dclose(d);
    set_err("HDF5 dataset %s: %lld elements, expected %lld", path, n, expect);
    return CLOUDSC_EIO;
  }
  herr_t e = H5.dread(d, as_int ? *H5.native_int : *H5.native_double, H5S_ALL_, H5S_ALL_, H5P_DEFAULT_, buf);
  H5.dclose(d);
  if (e < 0) { set_err("HDF5 read of %s failed", path); return CLOUDSC_EIO; }
  return CLOUDSC_OK;
}

static int h5_exists(hid_t file, const char *name) {
  char path[160];
  snprintf(path, sizeof(path), "/%s", name);
  hid_t d = H5.dopen2(file, path, H5P_DEFAULT_);
  if (d < 0) return 0;
  H5.dclose(d);
  return 1;
}

int cloudsc_io_load_hdf5_reference(const char *reference_h5, cloudsc_dataset_t *ds) {
  if (!reference_h5 || !ds || ds->klon <= 0) return CLOUDSC_EINVAL;
  if (!h5_load()) return CLOUDSC_EIO;
  for (int i = 0; i < CLOUDSC_NVALID; i++) { free(ds->ref[i]); ds->ref[i] = NULL; }
  ds->has_reference = 0;
  int rc = CLOUDSC_OK;
  hid_t r = H5.fopen(reference_h5, H5F_ACC_RDONLY_, H5P_DEFAULT_);
  if (r < 0) { set_err("cannot open %s read-only", reference_h5); return CLOUDSC_EIO; }
  int klon = 0, klev = 0;
  rc = h5_read(r, "KLON", 1, 1, &klon);
  if (!rc) rc = h5_read(r, "KLEV", 1, 1, &klev);
  if (!rc && (klon != ds->klon || klev != ds->klev)) {
    set_err("%s: KLON/KLEV %d/%d differ from the input's %d/%d", reference_h5, klon, klev, ds->klon, ds->klev);
    rc = CLOUDSC_EIO;
  }
  for (int i = 0; !rc && i < CLOUDSC_NVALID; i++) {
    const long long ne = cloudsc_io_elems(cloudsc_io_ref_kind[i], ds->klev, ds->klon);
    ds->ref[i] = (double *)malloc((size_t)ne * sizeof(double));
    if (!ds->ref[i]) { rc = CLOUDSC_ENOMEM; break; }
    rc = h5_read(r, cloudsc_io_ref_names[i], ne, 0, ds->ref[i]);
  }
  H5.fclose(r);
  if (rc) {
    for (int i = 0; i < CLOUDSC_NVALID; i++) { free(ds->ref[i]); ds->ref[i] = NULL; }
    return rc;
  }
  ds->has_reference = 1;
  return CLOUDSC_OK;
}

int cloudsc_io_load_hdf5(const char *input_h5, const char *reference_h5, cloudsc_dataset_t *ds) {
  if (!input_h5 || !ds) return CLOUDSC_EINVAL;
  if (!check_layout()) { set_err("cloudsc_params_t layout mismatch"); return CLOUDSC_EINVAL; }
  memset(ds, 0, sizeof(*ds));
  if (!h5_load()) return CLOUDSC_EIO;
  hid_t f = H5.fopen(input_h5, H5F_ACC_RDONLY_, H5P_DEFAULT_);
  if (f < 0) { set_err("cannot open %s read-only", input_h5); return CLOUDSC_EIO; }
  int rc = h5_read(f, "KLON", 1, 1, &ds->klon);
  if (!rc) rc = h5_read(f, "KLEV", 1, 1, &ds->klev);
  if (!rc && (ds->klon <= 0 || ds->klev < 2)) { set_err("%s: bad KLON/KLEV", input_h5); rc = CLOUDSC_EIO; }
  for (int i = 0; !rc && i < CLOUDSC_IO_NIN; i++) {
    const long long ne = cloudsc_io_elems(cloudsc_io_input_kind[i], ds->klev, ds->klon);
    if (i >= CLOUDSC_IO_FIRST_AEROSOL && !h5_exists(f, cloudsc_io_input_names[i])) continue;
    void *buf = malloc((size_t)ne * (i == CLOUDSC_IO_KTYPE ? sizeof(int) : sizeof(double)));
    if (!buf) { rc = CLOUDSC_ENOMEM; break; }
    if (i == CLOUDSC_IO_KTYPE) ds->ktype = (int *)buf;
    else ds->in[i] = (double *)buf;
    rc = h5_read(f, cloudsc_io_input_names[i], ne, i == CLOUDSC_IO_KTYPE, buf);
  }
  for (int i = 0; !rc && i < N_PDOUBLE; i++)
    rc = h5_read(f, k_param_double_names[i], 1, 0, &param_doubles(&ds->params)[i]);
  for (int i = 0; !rc && i < N_PINT; i++)
    rc = h5_read(f, k_param_int_names[i], 1, 1, &param_ints(&ds->params)[i]);
  H5.fclose(f);
  if (!rc && reference_h5) rc = cloudsc_io_load_hdf5_reference(reference_h5, ds);
  if (rc) { cloudsc_io_free(ds); return rc; }
  snprintf(ds->source, sizeof(ds->source), "HDF5 %s%s%s (read-only)", input_h5, reference_h5 ? " + " : "",
           reference_h5 ? reference_h5 : "");
  return CLOUDSC_OK;
}

/* write one dataset: dims of rank nd, element type file_t / mem_t */
static int h5_write(hid_t f, const char *name, int nd, const hsize_t *dims, hid_t file_t, hid_t mem_t,
                    const void *buf) {
  char path[160];
  snprintf(path, sizeof(path), "/%s", name);
  hid_t s = H5.s_create_simple(nd, dims, NULL);
  if (s < 0) { set_err("H5Screate_simple(%s) failed", path); return CLOUDSC_EIO; }
  hid_t d = H5.dcreate2(f, path, file_t, s, H5P_DEFAULT_, H5P_DEFAULT_, H5P_DEFAULT_);
  herr_t e = d >= 0 ? H5.dwrite(d, mem_t, H5S_ALL_, H5S_ALL_, H5P_DEFAULT_, buf) : -1;
  if (d >= 0) H5.dclose(d);
  H5.sclose(s);
  if (e < 0) { set_err("HDF5 write of %s failed", path); return CLOUDSC_EIO; }
  return CLOUDSC_OK;
}

static void kind_dims(int kind, int klev, int klon, int *nd, hsize_t *dims) {
  switch (kind) {
    case 0: *nd = 2; dims[0] = klev; dims[1] = klon; break;
    case 1: *nd = 2; dims[0] = klev + 1; dims[1] = klon; break;
    case 2: *nd = 3; dims[0] = CLOUDSC_NCLV; dims[1] = klev; dims[2] = klon; break;
    default: *nd = 1; dims[0] = klon; break;
  }
}

static int write_dims(hid_t f, const cloudsc_dataset_t *ds) {
  const hsize_t one = 1;
  long long v = ds->klon;
  int rc = h5_write(f, "KLON", 1, &one, *H5.std_i64le, *H5.native_llong, &v);
  v = ds->klev;
  if (!rc) rc = h5_write(f, "KLEV", 1, &one, *H5.std_i64le, *H5.native_llong, &v);
  v = 0;   /* extra diagnostic fields (ZBUDCC(KLON,KFLDX)): none, as in config-files/reference.h5 */
  if (!rc) rc = h5_write(f, "KFLDX", 1, &one, *H5.std_i64le, *H5.native_llong, &v);
  return rc;
}

int cloudsc_io_write_hdf5(const cloudsc_dataset_t *ds, const char *input_h5, const char *reference_h5) {
  if (!ds) return CLOUDSC_EINVAL;
  if (!h5_load()) return CLOUDSC_EIO;
  int rc = CLOUDSC_OK;
  if (input_h5) {
    hid_t f = H5.fcreate(input_h5, H5F_ACC_TRUNC_, H5P_DEFAULT_, H5P_DEFAULT_);
    if (f < 0) { set_err("cannot create %s", input_h5); return CLOUDSC_EIO; }
    rc = write_dims(f, ds);
    for (int i = 0; !rc && i < CLOUDSC_IO_NIN; i++) {
      int nd;
      hsize_t dims[3];
      kind_dims(cloudsc_io_input_kind[i], ds->klev, ds->klon, &nd, dims);
      if (i == CLOUDSC_IO_KTYPE)
        rc = h5_write(f, "KTYPE", nd, dims, *H5.std_i32le, *H5.native_int, ds->ktype);
      else if (ds->in[i])
        rc = h5_write(f, cloudsc_io_input_names[i], nd, dims, *H5.ieee_f64le, *H5.native_double, ds->in[i]);
    }
    const hsize_t one = 1;
    for (int i = 0; !rc && i < N_PDOUBLE; i++)
      rc = h5_write(f, k_param_double_names[i], 1, &one, *H5.ieee_f64le, *H5.native_double,
                    &cparam_doubles(&ds->params)[i]);
    for (int i = 0; !rc && i < N_PINT; i++)
      rc = h5_write(f, k_param_int_names[i], 1, &one, *H5.std_i32le, *H5.native_int,
                    &cparam_ints(&ds->params)[i]);
    H5.fclose(f);
    if (rc) return rc;
  }
  if (reference_h5) {
    if (!ds->has_reference) { set_err("dataset has no reference outputs"); return CLOUDSC_EINVAL; }
    hid_t f = H5.fcreate(reference_h5, H5F_ACC_TRUNC_, H5P_DEFAULT_, H5P_DEFAULT_);
    if (f < 0) { set_err("cannot create %s", reference_h5); return CLOUDSC_EIO; }
    rc = write_dims(f, ds);
    for (int i = 0; !rc && i < CLOUDSC_NVALID; i++) {
      int nd;
      hsize_t dims[3];
      kind_dims(cloudsc_io_ref_kind[i], ds->klev, ds->klon, &nd, dims);
      rc = h5_write(f, cloudsc_io_ref_names[i], nd, dims, *H5.ieee_f64le, *H5.native_double, ds->ref[i]);
    }
    H5.fclose(f);
  }
  return rc;
}

/* ------------------------------------------------------------------------ */
/* views for the C ABI                                                       */
/* ------------------------------------------------------------------------ */
void cloudsc_io_template(const cloudsc_dataset_t *ds, cloudsc_template_t *t) {
  memset(t, 0, sizeof(*t));
  t->klon = ds->klon;
  t->klev = ds->klev;
  const double *const *in = (const double *const *)ds->in;
  t->pt = in[0]; t->pq = in[1]; t->tendency_tmp_t = in[2]; t->tendency_tmp_q = in[3];
  t->tendency_tmp_a = in[4]; t->tendency_tmp_cld = in[5]; t->pvfl = in[6]; t->pvfi = in[7];
  t->phrsw = in[8]; t->phrlw = in[9]; t->pvervel = in[10]; t->pap = in[11]; t->paph = in[12];
  t->plsm = in[13]; t->ktype = ds->ktype; t->plu = in[15]; t->plude = in[16]; t->psnde = in[17];
  t->pmfu = in[18]; t->pmfd = in[19]; t->pa = in[20]; t->pclv = in[21]; t->psupsat = in[22];
  t->plcrit_aer = in[23]; t->picrit_aer = in[24]; t->pre_ice = in[25]; t->pccn = in[26]; t->pnice = in[27];
}

void cloudsc_io_reference(const cloudsc_dataset_t *ds, cloudsc_reference_t *r) {
  r->klon = ds->klon;
  r->klev = ds->klev;
  for (int i = 0; i < CLOUDSC_NVALID; i++) r->field[i] = ds->ref[i];
}

/* ------------------------------------------------------------------------ */
/* host block layout: expansion and statistics                               */
/* ------------------------------------------------------------------------ */
static int kind_nlev(int kind, int klev) {
  return kind == 0 ? klev : kind == 1 ? klev + 1 : kind == 2 ? CLOUDSC_NCLV * klev : 1;
}

void cloudsc_io_expand(const void *src, int kind, int is_int, int klev, int klon, int ngptot, int nproma,
                       long long col_offset, int elem_size, void *dst) {
  const int nlev = kind_nlev(kind, klev);
  const long long nb = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  for (long long b = 0; b < nb; b++)
    for (int l = 0; l < nlev; l++)
      for (int i = 0; i < nproma; i++) {
        const long long g = col_offset + b * nproma + i;
        const size_t s = (size_t)l * klon + (size_t)(g % klon);
        const size_t d = ((size_t)b * nlev + l) * nproma + i;
        if (is_int) ((int *)dst)[d] = ((const int *)src)[s];
        else if (elem_size == 8) ((double *)dst)[d] = ((const double *)src)[s];
        else ((float *)dst)[d] = (float)((const double *)src)[s];
      }
}

/* (hi, lo) += x as a double-double (TwoSum + renormalisation), the same
 * arithmetic as the device statistics (cloudsc_state.hip, dd_add) */
static void dd_acc(double *hi, double *lo, double x) {
  const double s = *hi + x, bb = s - *hi;
  const double e = (*hi - (s - bb)) + (x - bb);
  const double t = e + *lo;
  const double h = s + t;
  *lo = t - (h - s);
  *hi = h;
}

void cloudsc_io_field_stats(const double *ref, int kind, int klev, int klon, const void *field, int elem_size,
                            int ngptot, int nproma, long long col_offset, cloudsc_stats_t *st) {
  const int nlev = kind_nlev(kind, klev);
  const long long nb = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  double mn = DBL_MAX, mx = -DBL_MAX, me = 0.0;
  double es = 0.0, es_lo = 0.0, rs = 0.0, rs_lo = 0.0;   /* double-double sums, as the device statistics */
  for (long long b = 0; b < nb; b++) {
    const long long bsize = ngptot - b * nproma < nproma ? ngptot - b * nproma : nproma;
    for (int l = 0; l < nlev; l++)
      for (long long i = 0; i < bsize; i++) {
        const long long g = col_offset + b * nproma + i;
        const size_t d = ((size_t)b * nlev + l) * nproma + (size_t)i;
        const double v = elem_size == 8 ? ((const double *)field)[d] : (double)((const float *)field)[d];
        const double r = ref[(size_t)l * klon + (size_t)(g % klon)];
        const double df = fabs(v - r);
        mn = fmin(mn, v); mx = fmax(mx, v); me = fmax(me, df);
        dd_acc(&es, &es_lo, df);
        dd_acc(&rs, &rs_lo, fabs(r));
      }
  }
  st->minval = mn; st->maxval = mx; st->maxerr = me; st->errsum = es; st->refsum = rs;
  st->errsum_lo = es_lo; st->refsum_lo = rs_lo;
}

int cloudsc_io_load_dir(const char *dir, int with_reference, cloudsc_dataset_t *ds) {
  if (!dir || !ds) return CLOUDSC_EINVAL;
  char path[1024];
  snprintf(path, sizeof(path), "%s/MetaData-input.json", dir);
  return file_exists(path) ? cloudsc_io_load_serialbox(dir, with_reference, ds)
                           : cloudsc_io_load_raw(dir, with_reference, ds);
}
