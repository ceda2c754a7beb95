// cloudsc_internal.h -- host-side internals shared by the translation units of
// libcloudsc_amd.so (kernels + low-level ABI, device-resident state, host
// pipeline).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "cloudsc_amd.h"

namespace cloudsc_impl {

constexpr int kMaxDevices = 64;

// records "what: hip error string" for cloudsc_last_hip_error(); returns CLOUDSC_EHIP
int hip_fail(hipError_t e, const char* what);
// sets the cloudsc_last_hip_error() text for a failure that is not a HIP error
void set_error_text(const char* text);
// device / precision / variant / size checks shared by every entry point
int validate_run_args(int device, int precision, int variant, int ngptot, int nproma, int klev);
// every pointer the kernel reads or writes (aerosol inputs excepted) is set
bool fields_complete(const cloudsc_fields_t* f);
// cloudsc_gpu_run with an optional separate source of plude (NULL = in place)
int gpu_run_impl(int device, void* stream, int precision, int variant, int ngptot, int nproma, int klev,
                 const cloudsc_fields_t* f, void* scratch, const void* plude_in);

}  // namespace cloudsc_impl

#define HIPCHK(call)                                                \
  do {                                                              \
    hipError_t e_ = (call);                                         \
    if (e_ != hipSuccess) return cloudsc_impl::hip_fail(e_, #call); \
  } while (0)
