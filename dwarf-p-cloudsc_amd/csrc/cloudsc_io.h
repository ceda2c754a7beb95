/*
 * cloudsc_io.h -- dataset plumbing of the dwarf host driver (C, no GPU).
 *
 * Loads the KLON-column input state, the parameter block and the KLON-column
 * reference outputs that the reference driver reads (src/cloudsc_c/cloudsc/
 * load_state.c:45-66 dimensions, :279-690 inputs + scalars, :694-800
 * reference), from either
 *   - HDF5 (input.h5 / reference.h5, the reference's own format; dataset per
 *     field, C-order [lev][klon] / [nclv][lev][klon] / [klon], scalars as
 *     1-element datasets "/PTSPHY", "/RG", "/YRECLDP_<NAME>" ...).  libhdf5 is
 *     dlopen'ed at run time and files are opened READ-ONLY (the C reference
 *     opens them H5F_ACC_RDWR, load_state.c:60,499,746, which fails on a
 *     read-only reference.h5; the Fortran reader is read-only,
 *     hdf5_file_mod.F90:98-100), or
 *   - a raw directory (input_<NAME>.dat / reference_<NAME>.dat: the Serialbox
 *     binary arrays of the reference's data/, plus params.txt and
 *     manifest.json), used when no HDF5 library or file is available.
 *
 * Also writes input.h5 / reference.h5 from a loaded dataset (the input.h5
 * regeneration tool: the reference ships only reference.h5).
 */
#ifndef CLOUDSC_IO_H
#define CLOUDSC_IO_H

#include "cloudsc_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* input fields of the template, in cloudsc_template_t order */
#define CLOUDSC_IO_NIN 28
typedef struct cloudsc_dataset {
  int klon, klev;
  cloudsc_params_t params;
  /* template arrays (double, except ktype); NULL when absent (aerosols) */
  double *in[CLOUDSC_IO_NIN];      /* index: cloudsc_io_input_names order */
  int *ktype;
  /* reference outputs, cloudsc_field_id order; NULL when not loaded */
  double *ref[CLOUDSC_NVALID];
  int has_reference;
  char source[512];                /* what was read, for the log */
} cloudsc_dataset_t;

/* Upper-case dataset / file names: inputs (KTYPE is index CLOUDSC_IO_KTYPE). */
extern const char *const cloudsc_io_input_names[CLOUDSC_IO_NIN];
#define CLOUDSC_IO_KTYPE 14
/* field kind: 0 = [lev][klon], 1 = [lev+1][klon], 2 = [nclv][lev][klon], 3 = [klon] */
extern const int cloudsc_io_input_kind[CLOUDSC_IO_NIN];
/* aerosol inputs (optional) are the last five */
#define CLOUDSC_IO_FIRST_AEROSOL 23
/* HDF5 / file names of the 21 validated fields (cloudsc_field_id order) and
 * the names the dwarf prints (cloudsc_validate.c:195-215) */
extern const char *const cloudsc_io_ref_names[CLOUDSC_NVALID];
extern const char *const cloudsc_io_print_names[CLOUDSC_NVALID];
extern const int cloudsc_io_ref_kind[CLOUDSC_NVALID];

long long cloudsc_io_elems(int kind, int klev, int klon);

/* Load from a raw directory.  Returns CLOUDSC_OK or CLOUDSC_EIO / ENOMEM. */
int cloudsc_io_load_raw(const char *dir, int with_reference, cloudsc_dataset_t *ds);

/* Load from a Serialbox store -- the reference's own data/ directory:
 * MetaData-input.json (KLON/KLEV + parameters in global_meta_info, dims and
 * types in field_map), ArchiveMetaData-input.json (offsets) and
 * input_<FIELD>.dat; reference outputs from the "reference" prefix. */
int cloudsc_io_load_serialbox(const char *dir, int with_reference, cloudsc_dataset_t *ds);

/* A data directory: a Serialbox store if it holds MetaData-input.json, else
 * the raw form (manifest.json + params.txt). */
int cloudsc_io_load_dir(const char *dir, int with_reference, cloudsc_dataset_t *ds);

/* Load from HDF5 files (reference_h5 may be NULL).  CLOUDSC_EIO if libhdf5
 * cannot be loaded or a file / dataset is missing; errors are described in
 * cloudsc_io_last_error(). */
int cloudsc_io_load_hdf5(const char *input_h5, const char *reference_h5, cloudsc_dataset_t *ds);

/* Replace the dataset's reference outputs by those of a reference.h5
 * (KLON/KLEV must match). */
int cloudsc_io_load_hdf5_reference(const char *reference_h5, cloudsc_dataset_t *ds);

/* Write the dataset's inputs + scalars as input.h5, and/or its reference
 * outputs as reference.h5 (either path may be NULL). */
int cloudsc_io_write_hdf5(const cloudsc_dataset_t *ds, const char *input_h5, const char *reference_h5);

/* 1 if a libhdf5 could be dlopen'ed (CLOUDSC_HDF5_LIB, libhdf5.so, ...). */
int cloudsc_io_hdf5_available(void);

void cloudsc_io_free(cloudsc_dataset_t *ds);

/* Views of a loaded dataset for the C ABI (no copies). */
void cloudsc_io_template(const cloudsc_dataset_t *ds, cloudsc_template_t *t);
void cloudsc_io_reference(const cloudsc_dataset_t *ds, cloudsc_reference_t *r);

/* Host-side block layout (for the host-buffer path): expand template array
 * `src` of kind (0 level, 1 half level, 2 species, 3 surface) into dst
 * [nblocks][..][nproma] with the global map g % klon, g = col_offset + b*nproma + i
 * (load_state.c:69-184; lanes past ngptot are filled the same way, like the C
 * reference).  elem_size 8 (double), 4 (float, rounded from double) or 4 with
 * is_int (int copy). */
void cloudsc_io_expand(const void *src, int kind, int is_int, int klev, int klon, int ngptot, int nproma,
                       long long col_offset, int elem_size, void *dst);

/* ERROR_PRINT statistics (validate_mod.F90:118-146, fabs) of a block-layout
 * field (double or float, elem_size 8/4) against a KLON-column template
 * reference, over the ngptot active lanes. */
void cloudsc_io_field_stats(const double *ref, int kind, int klev, int klon, const void *field, int elem_size,
                            int ngptot, int nproma, long long col_offset, cloudsc_stats_t *st);

const char *cloudsc_io_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* CLOUDSC_IO_H */
