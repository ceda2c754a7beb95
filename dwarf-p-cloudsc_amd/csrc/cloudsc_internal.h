// cloudsc_internal.h -- host-side internals shared by the translation units of
// libcloudsc_amd.so (kernels + low-level ABI, device-resident state, host
// pipeline).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>

#include "cloudsc_amd.h"

namespace cloudsc_impl {

constexpr int kMaxDevices = 64;

// The fields of cloudsc_fields_t: shape kind, direction, element type, in
// member order (include/cloudsc_amd.h).
enum FieldKind { FK_LEVEL, FK_HALF, FK_SPECIES, FK_SURFACE };
enum FieldDir { FD_IN, FD_INOUT, FD_OUT, FD_AEROSOL };
struct FieldDesc { int kind, dir, is_int; };
// cloudsc_fields_t member order (include/cloudsc_amd.h)
inline constexpr FieldDesc kFieldTable[] = {
    {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_IN, 0},   {FK_SPECIES, FD_IN, 0}, {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_HALF, FD_IN, 0},    {FK_SURFACE, FD_IN, 0}, {FK_SURFACE, FD_IN, 1}, {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},   {FK_LEVEL, FD_IN, 0},
    {FK_SPECIES, FD_IN, 0}, {FK_LEVEL, FD_IN, 0},
    {FK_LEVEL, FD_AEROSOL, 0}, {FK_LEVEL, FD_AEROSOL, 0}, {FK_LEVEL, FD_AEROSOL, 0},
    {FK_LEVEL, FD_AEROSOL, 0}, {FK_LEVEL, FD_AEROSOL, 0},
    {FK_LEVEL, FD_INOUT, 0},
    {FK_LEVEL, FD_OUT, 0},  {FK_LEVEL, FD_OUT, 0},  {FK_LEVEL, FD_OUT, 0},  {FK_SPECIES, FD_OUT, 0},
    {FK_LEVEL, FD_OUT, 0},  {FK_SURFACE, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0},
    {FK_HALF, FD_OUT, 0},   {FK_HALF, FD_OUT, 0}};
inline constexpr int kNumFields = (int)(sizeof(kFieldTable) / sizeof(kFieldTable[0]));
static_assert(sizeof(cloudsc_fields_t) == kNumFields * sizeof(void*), "field table out of sync with the header");

inline size_t per_block_elems(int kind, int nproma, int klev) {
  switch (kind) {
    case FK_LEVEL: return (size_t)klev * nproma;
    case FK_HALF: return (size_t)(klev + 1) * nproma;
    case FK_SPECIES: return (size_t)CLOUDSC_NCLV * klev * nproma;
    default: return (size_t)nproma;
  }
}


// One parameter set on one device: the host-folded fp64 and fp32 DevParams
// blocks in device memory (read by the kernels through a KArgs pointer), plus
// the host-side values the launch itself needs.
struct ParamSet {
  void* dev = nullptr;     // device block (fp64 mirror at 0, fp32 mirror after it)
  int device = -1;
  bool aer = false;        // LAERICESED || LAERICEAUTO: aerosol inputs are read
  int ncldtop = 0;         // NCLDTOP (KSEG segment bounds)
};
int check_params(const cloudsc_params_t* p);
// (re)upload `p` into ps (allocated on first use) on `device`; synchronous
int param_set_upload(ParamSet* ps, int device, const cloudsc_params_t* p);
// copy of another set on the same device (device-to-device)
int param_set_copy(ParamSet* dst, const ParamSet* src);
void param_set_free(ParamSet* ps);
// the device's default set (cloudsc_gpu_init), NULL if never initialised
const ParamSet* device_default_params(int device);

// records "what: hip error string" for cloudsc_last_hip_error(); returns CLOUDSC_EHIP
int hip_fail(hipError_t e, const char* what);
// sets the cloudsc_last_hip_error() text for a failure that is not a HIP error
void set_error_text(const char* text);
// device / precision / variant / size checks shared by every entry point
int validate_run_args(int device, int precision, int variant, int ngptot, int nproma, int klev);
// every pointer the kernel reads or writes (aerosol inputs excepted) is set
bool fields_complete(const cloudsc_fields_t* f);
// Host record of one KSEG workspace owned by a caller that launches on it in
// stream order (a state): after the first launch zeroes it, later launches
// continue its ticket counter and flag stamps instead of zeroing it again.
struct KsegEpoch {
  bool ready = false;       // false: zero the workspace before the next launch
  unsigned base[8] = {};    // per dequeue stripe (kKsegStripes, cloudsc_kcache.h)
  unsigned stamp = 0;
};
// Start/stop events of one launch, recorded by the kernel's own dispatch
// (hipExtLaunchKernelGGL) instead of separate event packets around it.
struct LaunchEvents {
  hipEvent_t start, stop;
};
// cloudsc_gpu_run with an optional separate source of plude (NULL = in place),
// an explicit parameter set (NULL = the device's default set), an optional
// KSEG workspace record (NULL = zero the workspace before every KSEG launch)
// and optional events timing the physics kernel (NULL = none)
int gpu_run_impl(int device, void* stream, int precision, int variant, int ngptot, int nproma, int klev,
                 const cloudsc_fields_t* f, void* scratch, const void* plude_in, const ParamSet* ps,
                 KsegEpoch* ep = nullptr, const LaunchEvents* lev = nullptr);
// the kernel variant of a `variant` argument without its option bits (CLOUDSC_FP32_EXACT_LIBM)
inline int variant_kind(int variant) { return variant & 0xff; }
// waits for `stream` and returns CLOUDSC_EHANDOFF if the last KSEG launch on
// `scratch` counted a timed-out segment hand-off
int kseg_check(int device, void* stream, void* scratch);
// waits for `stream`; the effective shader clock of the KSEG launches on
// `scratch` since the last reset (sum of shader-clock cycles over sum of
// real-time ticks of the workgroups, times the real-time rate) and the summed
// workgroup-seconds behind it; reset zeroes the sums
int kseg_clock(int device, void* stream, void* scratch, bool reset, double* ghz, double* seconds);

// the memory-pattern probe of cloudsc_place.hip over f on `stream`: best of
// `reps` timed launches after one untimed, ms; mode 0 outputs written only, 1
// inputs read too (every non-NULL output of f is overwritten); strides (6, may
// be NULL): the inputs' and outputs' block / row / species element strides of
// another layout (cloudsc_debug_memory_probe_layout)
int memory_probe(int device, hipStream_t stream, int precision, int ngptot, int nproma, int klev,
                 const cloudsc_fields_t* f, int mode, int reps, hipEvent_t e0, hipEvent_t e1, float* best_ms,
                 const long long* strides = nullptr);

// What a placement search cost and found (cloudsc_place.hip)
struct PlaceCost {
  float first_ms = 0.f, final_ms = 0.f;   // probe time of the first / the kept placement
  int tries = 0, moves = 0;               // candidate buffers allocated / kept
  int launches = 0;                       // probe launches (untimed ones included)
  double search_ms = 0.0;                 // wall time of the search
  long long peak_bytes = 0;               // most candidate and spacer bytes held at once
  long long budget_bytes = 0;             // the bound search_fits was asked for (peak_bytes stays below it)
};
// the output placement search (see cloudsc_place.hip): moves f's output
// members (members/bytes: positions in cloudsc_fields_t and sizes) to the
// fastest candidate buffers under `probe` (ms, < 0 on an error); never frees
// the caller's original buffers
int search_outputs(cloudsc_fields_t& f, const int* members, const size_t* bytes, int n, int sets, int passes,
                   uint32_t seed, const std::function<float(const cloudsc_fields_t&)>& probe, PlaceCost& cost);

// Device allocations of the state and the placement searches.  Plain
// hipMalloc / hipExtMallocWithFlags + hipFree; in the diagnostic build
// -DCLOUDSC_DEBUG_CANARY every buffer gets a 64 KiB guard band of a known byte
// on each side, checked by cloudsc_debug_canary_check and at free (the
// round-5 record of the contiguous-allocation failure).
hipError_t dev_malloc(void** p, size_t bytes, unsigned flags = 0);
void dev_free(void* p);

// whether a placement search whose candidates peak at about `transient` bytes
// fits the device's free memory with room to spare (on a device
// shared by several ranks the search must not starve their allocations)
bool search_fits(size_t transient);
// the transient bytes a placement search holds at most over sets of set_bytes
// in n buffers with `sets` whole sets tried: two candidate sets and the spacers
size_t search_transient_bytes(size_t set_bytes, int n, int sets);

// copy ceiling on the pipelines' engine pair (cloudsc_pipeline.hip)
int pcie_engine_gbps(int device, size_t nb, int reps, double* h2d, double* d2h, double* both);

}  // namespace cloudsc_impl

#define HIPCHK(call)                                                \
  do {                                                              \
    hipError_t e_ = (call);                                         \
    if (e_ != hipSuccess) return cloudsc_impl::hip_fail(e_, #call); \
  } while (0)
