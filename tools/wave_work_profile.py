#!/usr/bin/env python3
"""Diagnostic (host only): how many exp / pow / divisions a 64-column wave
executes per level on a given state, counting each call site once per
(wave, level) if ANY of its lanes reaches it -- the SIMT cost of divergent
branches -- next to the per-lane count.

Builds a patched copy of the phase functions (csrc/cloudsc_kcache.h through
the host path of cloudsc_cpu.hip) whose host cl_exp / cl_pow / cl_div record
their call site (__builtin_LINE()), runs 64-column blocks level by level, and
prints per call site: lane hits, wave-level hits, and the totals per level.

usage: wave_work_profile.py [ngptot] [scenario: ref|W|M]"""
import ctypes as C
import os
import re
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import cloudsc_amd as ca  # noqa: E402

TMP = "/tmp/wave_work_profile"


def build():
    shutil.rmtree(TMP, ignore_errors=True)
    shutil.copytree(os.path.join(REPO, "dwarf-p-cloudsc_amd", "csrc"), os.path.join(TMP, "csrc"))
    dev = os.path.join(TMP, "csrc", "cloudsc_dev.h")
    s = open(dev).read()
    hook = '''
namespace cloudsc {
extern "C" void wwp_hit(int kind, int line);
}
'''
    s = s.replace("namespace cloudsc {\n", hook + "namespace cloudsc {\n", 1)
    s = s.replace("template <typename real>\nCLOUDSC_HD real cl_pow(real x, real y) {\n#if defined(__HIP_DEVICE_COMPILE__)",
                  "template <typename real>\nCLOUDSC_HD real cl_pow(real x, real y, int line_ = __builtin_LINE()) {\n"
                  "#if !defined(__HIP_DEVICE_COMPILE__)\n  wwp_hit(1, line_);\n#endif\n#if defined(__HIP_DEVICE_COMPILE__)")
    s = s.replace("template <typename real>\nCLOUDSC_HD real cl_exp(real x) {\n#if defined(__HIP_DEVICE_COMPILE__)",
                  "template <typename real>\nCLOUDSC_HD real cl_exp(real x, int line_ = __builtin_LINE()) {\n"
                  "#if !defined(__HIP_DEVICE_COMPILE__)\n  wwp_hit(0, line_);\n#endif\n#if defined(__HIP_DEVICE_COMPILE__)")
    s = s.replace("CLOUDSC_HD double cl_div(double n, double d) {\n#if !defined(__HIP_DEVICE_COMPILE__)\n",
                  "CLOUDSC_HD double cl_div(double n, double d, int line_ = __builtin_LINE()) {\n"
                  "#if !defined(__HIP_DEVICE_COMPILE__)\n  wwp_hit(2, line_);\n")
    s = s.replace("template <typename real>\nCLOUDSC_HD real cl_div(typename std::common_type<real>::type n, "
                  "typename std::common_type<real>::type d) {\n  return cl_div(static_cast<real>(n), static_cast<real>(d));",
                  "template <typename real>\nCLOUDSC_HD real cl_div(typename std::common_type<real>::type n, "
                  "typename std::common_type<real>::type d, int line_ = __builtin_LINE()) {\n"
                  "  return cl_div(static_cast<real>(n), static_cast<real>(d), line_);")
    open(dev, "w").write(s)
    drv = os.path.join(TMP, "csrc", "wwp.hip")
    src = open(os.path.join(TMP, "csrc", "cloudsc_cpu.hip")).read()
    # per (level, column) bookkeeping: the cpu loop is level-outer, column-inner over a block
    src = src.replace('extern "C" int cloudsc_cpu_run(', 'extern "C" int cloudsc_cpu_run_unused(')
    src = src.replace("    for (int jl = 0; jl < bsize; jl++) {\n      const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);\n      HostColumn<real>& h = col[jl];\n      LevelIn<real> cur;",
                      "    wwp_level_begin();\n    for (int jl = 0; jl < bsize; jl++) {\n      const unsigned lo = (unsigned)jl * (unsigned)sizeof(real);\n      HostColumn<real>& h = col[jl];\n      LevelIn<real> cur;")
    src = src.replace("  for (int jl = 0; jl < bsize; jl++) stg(A.prainfrac",
                      "  wwp_level_begin();\n  for (int jl = 0; jl < bsize; jl++) stg(A.prainfrac")
    src = src.replace("namespace {\n\n// The state of one column",
                      '''static long long g_lane[3][4096], g_wave[3][4096], g_levels;
static unsigned char g_seen[3][4096];
extern "C" void cloudsc::wwp_hit(int kind, int line) { g_lane[kind][line]++; g_seen[kind][line] = 1; }
static void wwp_level_begin() {
  for (int k = 0; k < 3; k++) for (int l = 0; l < 4096; l++) if (g_seen[k][l]) { g_wave[k][l]++; g_seen[k][l] = 0; }
  g_levels++;
}
extern "C" void wwp_result(long long* lane, long long* wave, long long* levels) {
  wwp_level_begin(); g_levels--;
  for (int k = 0; k < 3; k++) for (int l = 0; l < 4096; l++) { lane[k * 4096 + l] = g_lane[k][l]; wave[k * 4096 + l] = g_wave[k][l]; }
  *levels = g_levels;
}
namespace {

// The state of one column''')
    src += '''
extern "C" int wwp_run(int ngptot, int nproma, int klev, const cloudsc_params_t* params, const cloudsc_fields_t* f) {
  const DevParams<double> c = fold_params<double>(*params);
  const KArgs<double> A = host_args(f, ngptot, nproma, klev);
  const int nblocks = ngptot / nproma + (ngptot % nproma ? 1 : 0);
  std::vector<HostColumn<double>> col((size_t)nproma);
  for (int b = 0; b < nblocks; b++) run_block<double, false>(c, A, b, col);
  return 0;
}
'''
    open(drv, "w").write(src)
    out = os.path.join(TMP, "libwwp.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O1", "-ffp-contract=off", "-fPIC", "-std=c++17",
                           "--offload-arch=gfx950", "-Xarch_host", "-mfma", "-I" + os.path.join(REPO, "include"),
                           "-I" + os.path.join(TMP, "csrc"), "-shared", drv, "-o", out,
                           "-L" + os.path.join(REPO, "dwarf-p-cloudsc_amd"), "-lcloudsc_amd",
                           "-Wl,-rpath," + os.path.join(REPO, "dwarf-p-cloudsc_amd")])
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6400
    scen = sys.argv[2] if len(sys.argv) > 2 else "ref"
    lib = C.CDLL(build())
    ds = ca.load_dataset()
    if scen != "ref":
        import make_fixtures as mf
        ds = mf.load_scenario(scen, ds)
    st = ca.make_host_state(ds, n, 64)
    p = ca.Params.from_dict(ds.params)
    f = st.fields()
    lib.wwp_run(n, 64, ds.klev, C.byref(p), C.byref(f))
    lane = (C.c_longlong * (3 * 4096))()
    wave = (C.c_longlong * (3 * 4096))()
    levels = C.c_longlong()
    lib.wwp_result(lane, wave, C.byref(levels))
    L = levels.value
    src = open(os.path.join(TMP, "csrc", "cloudsc_kcache.h")).read().splitlines()
    names = ["exp", "pow", "div"]
    tot_w = [0.0, 0.0, 0.0]
    tot_l = [0.0, 0.0, 0.0]
    print("state %s, %d columns, %d wave-levels (64 columns each)" % (scen, n, L))
    print("%-4s %5s %10s %10s  %s" % ("kind", "line", "lane/lvl", "wave/lvl", "source"))
    for k in range(3):
        for l in range(4096):
            if wave[k * 4096 + l]:
                wl = wave[k * 4096 + l] / L
                ll = lane[k * 4096 + l] / (L * 64.0)
                tot_w[k] += wl
                tot_l[k] += ll
                txt = src[l - 1].strip()[:70] if 0 < l <= len(src) else "(cloudsc_dev.h)"
                if wl > 0.02:
                    print("%-4s %5d %10.3f %10.3f  %s" % (names[k], l, ll, wl, txt))
    for k in range(3):
        print("TOTAL %s per wave-level: %.2f executed (SIMT), %.2f per lane" % (names[k], tot_w[k], tot_l[k]))


if __name__ == "__main__":
    main()
