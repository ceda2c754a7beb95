#!/usr/bin/env python3
"""CLOUDSC dwarf benchmark: grid-columns/sec at NGPTOT=163840 per GPU, KLEV=137,
fp64 (BASELINE.json metric), plus the HBM roofline of the k-caching kernel and
the CPU baseline measured on this box's host cores.

One process per GPU (launched by torch.distributed.run for N>1).  Columns shard
with NO data-path collective: rank r owns global columns
[r*NGPTOT, (r+1)*NGPTOT) (weak scaling, the g % 100 map of the GLOBAL index, so
a sharded run is bit-identical to an unsharded one).  torch.distributed (gloo)
is used only for the barrier around the timed region and the max-over-ranks.

A "step" = one CLOUDSC pass over the rank's NGPTOT resident columns: one
kernel launch reading every input (plude from the state's pristine copy: the
INOUT field is taken out of place, so repeated steps are the same step) and
writing every output.  The timed region brackets exactly K steps with barrier
+ device sync on both sides; value = all columns of all ranks / max-over-ranks
wall time.  The K launches are plain dispatches, timed as a whole by two HIP
events on the launch stream (cloudsc_state_run_span): roofline.achieved uses
that time / K.  A second, untimed pass of K launches, each recording its own
start/stop events in its dispatch packet (hipExtLaunchKernelGGL), gives the
per-launch distribution (kernel_ms_median / p10 / p90).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))

BYTES_PER_COL = {8: 56036, 4: 28020}     # SURVEY.md §8d algorithmic bytes per column
# of which read (inputs incl. plude and ktype): 3701 values + 4 B; written: 3303 values
IN_BYTES_PER_COL = {8: 3701 * 8 + 4, 4: 3701 * 4 + 4}
HBM_PEAK_GBS = 8000.0                    # MI355X HBM3E spec (MI355X_MICROARCH.md)
GUIDE_COPY_GBS = 6290.0                  # MI355X_MICROARCH.md:36, measured float4 copy (79 % of the spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)    # 0.2 s of kernels: a stable mean
    p.add_argument("--warmup", type=int, default=20,
                   help="minimum untimed steps; warm-up then continues by time until the per-launch kernel time "
                        "is stable (the board settles its shader clock over the first ~10-15 launches of the fp64 "
                        "kernel, profiles/r02/clock_probe_bench_run.json); the steps actually run are reported "
                        "as prewarm_steps")
    p.add_argument("--ngptot", type=int, default=163840, help="columns per GPU")
    p.add_argument("--nproma", type=int, default=64,
                   help="NPROMA (block = workgroup); 64 is the measured best for the persistent kernel "
                        "(profiles/r01/nproma_sweep_all_variants.jsonl)")
    p.add_argument("--precision", choices=["fp64", "fp32"], default="fp64")
    p.add_argument("--variant", choices=["kseg", "kcache", "scc", "scc-private"], default=None,
                   help="default: kseg (the persistent kernel: 2560 wave-sized units on 2 waves/SIMD without a "
                        "tail; fp64 and fp32, profiles/r02/kseg_grid_sweep.jsonl)")
    p.add_argument("--fp32-exact-libm", action="store_true",
                   help="fp32: exp/pow with the glibc algorithms (bit-identical to the fp32 restatement) instead of "
                        "the default float-internal device forms")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-transfer", action="store_true",
                   help="skip the host-buffer path (H2D -> kernel -> D2H, chunked over streams), which N=1 runs "
                        "by default and reports as pcie_inclusive -- the reference GPU drivers' TOTAL semantics "
                        "(cloudsc_driver.cu:344-456), never the headline value")
    p.add_argument("--transfer-steps", type=int, default=7)
    p.add_argument("--no-boundary", action="store_true",
                   help="skip the caller-owned-buffer leg (cloudsc_fields_alloc + cloudsc_gpu_run) that N=1 runs "
                        "and reports as boundary_path")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="host threads of the CPU baseline (default: OMP_NUM_THREADS, else all host cores)")
    p.add_argument("--no-hbm-peak", action="store_true", help="skip the in-run STREAM-copy measurement")
    p.add_argument("--energy-seconds", type=float, default=2.0,
                   help="after the timed region, run the kernel back to back this long while sampling the board's "
                        "power (hwmon) for energy_uj_per_column; 0 skips it")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                   help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    a = p.parse_args()
    if a.variant is None:
        a.variant = "kseg"
    return a


def prewarm_until_stable(g, variant, min_steps, np, batch=5, tol=0.005, floor=15, cap=400):
    """Untimed launches until the kernel time is stable: batches of `batch`
    launches, at least max(min_steps, floor) in all, until two consecutive batch
    medians agree within `tol` (the shader clock has settled), at most `cap`.
    Returns the number of launches run."""
    n, prev = 0, None
    need = max(min_steps, floor)
    while n < cap:
        m = float(np.median(g.run(variant, batch)))
        n += batch
        if n >= need and prev is not None and abs(m - prev) <= tol * prev:
            break
        prev = m
    return n


def cpu_baseline(ca, ds, nthreads):
    """BASELINE.md §4 on this box's host cores, rank 0 at N=1 only: the reference
    C kernel (oracle/_ref, compiled from src/cloudsc_c/cloudsc/cloudsc_c.c) in
    the C dwarf's OpenMP block loop, timed around the loop only
    (cloudsc_driver.c:181-231), at `1 16384 32` (config 1) and `T 163840 {16,32}`
    (T = the host threads of this box's share), each run validated against
    reference.h5 with the ERROR_PRINT statistics.  value = the faster of the two
    163840-column runs.  The library's own CPU variant (cloudsc_cpu_run) is timed
    beside it on the same states ("cpu_variant")."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle
    kind = "reference" if oracle.ref_available() else "port"
    eps10 = 10 * np.finfo(np.float64).eps
    runs, product = [], []
    for nth, ncols, nproma in ((1, 16384, 32), (nthreads, 163840, 16), (nthreads, 163840, 32)):
        st = ca.make_host_state(ds, ncols, nproma, ca.FP64)
        plude0 = st.arrays["plude"].copy()
        if kind == "reference":
            secs = oracle.run_ref_state(ds, st, nthreads=nth)
        else:
            _, secs = oracle.run_oracle(ds, ncols, nproma, nthreads=nth)
        worst = ca.validate_host_state(ds, st) if kind == "reference" else None
        runs.append({"cmd": "%d %d %d" % (nth, ncols, nproma), "columns_per_s": round(ncols / secs, 1),
                     "ms": round(1e3 * secs, 2), "worst_rel_l1": worst,
                     "validated": bool(worst is not None and worst <= eps10)})
        np.copyto(st.arrays["plude"], plude0)
        secs = ca.cpu_run_state(ds, st, nthreads=nth)
        w = ca.validate_host_state(ds, st)
        product.append({"cmd": "%d %d %d" % (nth, ncols, nproma), "columns_per_s": round(ncols / secs, 1),
                        "ms": round(1e3 * secs, 2), "worst_rel_l1": w, "validated": bool(w <= eps10)})
        del st, plude0
    full = [r for r in runs if r["cmd"].split()[1] == "163840"]
    best = max(full, key=lambda r: r["columns_per_s"])
    return {"value": best["columns_per_s"], "unit": "columns/s", "cores": nthreads, "kind": kind,
            "host": dict(host_cores(), threads_used=nthreads),
            "sample": "%s `%s` (163840 columns, the full workload; the faster NPROMA of 16/32), OpenMP block "
                      "loop timed like cloudsc_driver.c:181-231, validated vs reference.h5" % (
                          "reference kernel src/cloudsc_c/cloudsc/cloudsc_c.c compiled from its sources"
                          if kind == "reference" else "oracle restatement", best["cmd"]),
            "runs": runs,
            "cpu_variant": {"what": "this library's cloudsc_cpu_run (the GPU kernels' phase functions "
                                    "compiled for the host), same states", "runs": product}}


def launch_histogram(ms, np, width_us=10.0):
    """Counts of the per-launch times in `width_us` bins: {"lo_ms", "width_us", "counts"}."""
    a = np.asarray(ms, dtype=np.float64)
    lo = np.floor(a.min() * 1e3 / width_us) * width_us / 1e3
    idx = np.floor((a - lo) * 1e3 / width_us + 1e-9).astype(int)
    return {"lo_ms": round(float(lo), 4), "width_us": width_us,
            "counts": [int(c) for c in np.bincount(idx)]}


def host_cores():
    """The host CPU share the CPU baseline ran on: nproc (every CPU the machine
    has), the CPUs this process may run on (sched_getaffinity), the sockets and
    the model (from /sys and /proc/cpuinfo; best effort).  On the GPU pool the
    box's share is 16 threads (OMP_NUM_THREADS) of a much larger machine."""
    out = {"nproc": os.cpu_count(), "affinity_cpus": None, "sockets": None, "model": None,
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        aff = sorted(os.sched_getaffinity(0))
        out["affinity_cpus"] = len(aff)
        pk = set()
        for c in aff:
            try:
                pk.add(open("/sys/devices/system/cpu/cpu%d/topology/physical_package_id" % c).read().strip())
            except OSError:
                pass
        out["affinity_sockets"] = len(pk) or None
        allpk = set()
        for d in os.listdir("/sys/devices/system/cpu"):
            f = "/sys/devices/system/cpu/%s/topology/physical_package_id" % d
            if d.startswith("cpu") and d[3:].isdigit() and os.path.exists(f):
                allpk.add(open(f).read().strip())
        out["sockets"] = len(allpk) or None
    except (OSError, AttributeError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                out["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return out


def roofline_traffic(ca, path, key):
    """Per-launch HBM bytes from the committed rocprofv3 PMC passes, only if they
    were measured on the current kernel sources (kernel_source_hash)."""
    if not os.path.exists(path):
        return None, "no PMC measurement (%s)" % os.path.relpath(path, REPO)
    try:
        entry = json.load(open(path)).get(key)
    except Exception as e:            # an unreadable file is reported, not fatal
        return None, "unreadable %s: %s" % (path, e)
    if not entry:
        return None, "no PMC measurement for %s" % key
    if entry.get("kernel_source_hash") != ca.kernel_source_hash():
        return None, "PMC measurement is stale (measured on kernel sources %s, current %s)" % (
            entry.get("kernel_source_hash"), ca.kernel_source_hash())
    return entry["hbm_bytes_per_launch"], "rocprofv3 2xFETCH_SIZE+WRITE_SIZE per launch, kernel sources %s" % (
        entry["kernel_source_hash"])


def box_info():
    """The box's GPU memory / compute partition modes and memory clock range
    (rocm-smi queries, read-only; best effort): boxes of the pool run the same
    kernel at different speeds with a normal shader clock and STREAM rate
    (DESIGN.md section 7), and these are the first settings that could tell them apart."""
    import subprocess
    out = {}
    for key, flag in (("memory_partition", "--showmemorypartition"), ("compute_partition", "--showcomputepartition"),
                      ("mclk_range", "--showmclkrange")):
        try:
            r = subprocess.run(["rocm-smi", flag, "--json"], capture_output=True, text=True, timeout=20)
            d = json.loads(r.stdout) if r.returncode == 0 else {}
            cards = sorted(k for k in d if k.startswith("card"))
            out[key] = d[cards[0]] if cards else None
        except (OSError, ValueError, subprocess.SubprocessError):
            out[key] = None
    return out


def transfer_rate(ca, ds, args, prec, variant, chunk_blocks=128, slots=3):
    """Host-resident block-layout arrays (pinned in place), per chunk H2D ->
    kernel -> D2H pipelined over the two directions' copy engines and a kernel stream: the
    reference GPU drivers' TOTAL semantics (cloudsc_driver.cu:344-456).  plude
    is restored on the host between steps, outside the timed pipeline.  The
    default chunking is the measured best (profiles/r04/transfer_sweep_kseg_fp64.txt).
    Held against the box's copy ceiling measured here (cloudsc_pcie_gbps): the
    step moves in_bytes to the device and out_bytes back, so it takes at least
    max(in/h2d, out/d2h, (in+out)/both)."""
    pc = ca.pcie_gbps(0, 1 << 30, 3)
    hp = ca.HostPipeline(ds, args.ngptot, args.nproma, prec, chunk_blocks=chunk_blocks, nstreams=slots)
    try:
        mode, e_in, e_out = hp.copy_path()
        overlap, pairs = hp.engine_check()
        hp.run(variant)
        ms = [hp.run(variant) for _ in range(args.transfer_steps)]
        # the same step's copies without the kernels (same engines, arrays and slots), best of 3
        copy_ms = min(hp.copy_bound() for _ in range(3)) if mode == 1 else None
    finally:
        hp.close()
    # the median step: a single slow step (host-side page activity) would otherwise set the figure
    t = sorted(ms)[len(ms) // 2]
    es = 8 if prec == ca.FP64 else 4
    # per column: 23 level inputs + plude + aerosol-free species/half/surface inputs in, outputs + plude out
    # (the same algorithmic bytes as the roofline, split by direction: SURVEY.md §8d)
    in_b, out_b = IN_BYTES_PER_COL[es] * args.ngptot, (BYTES_PER_COL[prec] - IN_BYTES_PER_COL[es]) * args.ngptot
    probe_bound_ms = 1e3 * max(in_b / (pc["h2d"] * 1e9), out_b / (pc["d2h"] * 1e9),
                               (in_b + out_b) / (pc["both"] * 1e9))
    # the bound: the step's own copies without the kernels when measured (the probe's separate buffers
    # have shown a D2H rate of half the pipeline's own on one box), else the probe's rates
    bound_ms = copy_ms if copy_ms else probe_bound_ms
    return {"value": round(args.ngptot / (t * 1e-3), 1), "unit": "columns/s", "ms_per_step": round(t, 3),
            "ms_per_step_method": "median of the timed steps", "ms_per_step_mean": round(sum(ms) / len(ms), 3),
            "ms_per_step_min": round(min(ms), 3), "ms_per_step_all": [round(x, 2) for x in ms], "steps": len(ms),
            "chunk_blocks": chunk_blocks, "slots": slots,
            "copies": ("every copy on a copy engine of its own per direction (H2D engine mask 0x%x, D2H 0x%x), "
                       "ordered with the kernels from the host" % (e_in, e_out)) if mode == 1 else
                      "one H2D, one kernel, one D2H HIP stream (the runtime picks the copy engines)",
            "engine_check": {"overlap": round(overlap, 3), "pairs_tried": pairs,
                             "method": "at creation, 256 MiB each way at once / the slower direction alone on "
                                       "the engine pair (1.0 = fully concurrent); first pair under 1.3 kept"},
            "bytes_per_step": BYTES_PER_COL[prec] * args.ngptot, "bytes_in": in_b, "bytes_out": out_b,
            "copy_ceiling_gbs": {k: round(v, 1) for k, v in pc.items()},
            "bound_ms": round(bound_ms, 2), "frac_of_bound": round(bound_ms / t, 4),
            "bound_method": ("the same step's copies without the kernels on the same engines, host arrays and "
                             "device slots (cloudsc_host_pipeline_copy_bound), best of 3") if copy_ms else
                            "max(in/h2d, out/d2h, (in+out)/both) at the probe's rates",
            "probe_bound_ms": round(probe_bound_ms, 2),
            "note": "end-to-end TOTAL as the reference GPU drivers time it (H2D + kernel + D2H, "
                    "cloudsc_driver.cu:344,456), host-buffer path over PCIe; NOT the headline value"}


def boundary_path(ca, g, ds, args, prec, variant, np, launches=30):
    """The reference CUDA driver's shape on caller-owned buffers: every field
    allocated by cloudsc_fields_alloc (one buffer per field, the outputs placed
    by the memory-pattern search), the inputs copied in (from the state's buffers,
    device to device), the KSEG kernel launched through cloudsc_gpu_run on them,
    plude restored before each launch, HIP events on the null stream around each
    launch.  Reports the median kernel time and the search's cost beside the
    state's: what a caller of the low-level boundary gets."""
    import ctypes as C
    lib = ca.gpu_lib()
    hip = C.CDLL("libamdhip64.so")
    for fn, at in (("hipMalloc", [C.POINTER(C.c_void_p), C.c_size_t]), ("hipFree", [C.c_void_p]),
                   ("hipMemset", [C.c_void_p, C.c_int, C.c_size_t]), ("hipEventCreate", [C.POINTER(C.c_void_p)]),
                   ("hipEventRecord", [C.c_void_p, C.c_void_p]), ("hipEventSynchronize", [C.c_void_p]),
                   ("hipEventDestroy", [C.c_void_p]),
                   ("hipEventElapsedTime", [C.POINTER(C.c_float), C.c_void_p, C.c_void_p])):
        getattr(hip, fn).argtypes = at
    sf = ca.Fields()
    ca.check(lib.cloudsc_state_fields(g.h, C.byref(sf)))
    p = ca.Params.from_dict(ds.params)
    ca.check(lib.cloudsc_gpu_init(0, C.byref(p)))
    df = ca.DeviceFields(args.ngptot, args.nproma, ds.klev, prec)
    ws, e0, e1 = C.c_void_p(), C.c_void_p(), C.c_void_p()
    try:
        df.copy_from(sf, list(ca.INPUT_FIELDS))
        nb = lib.cloudsc_gpu_scratch_bytes(prec, variant, args.ngptot, args.nproma, ds.klev)
        assert hip.hipMalloc(C.byref(ws), nb) == 0 and hip.hipMemset(ws, 0, 256) == 0
        hip.hipEventCreate(C.byref(e0))
        hip.hipEventCreate(C.byref(e1))
        ms = []
        for i in range(launches + 5):
            ca.check(lib.cloudsc_state_reset(g.h))   # the state's plude buffer <- its pristine input
            ca.check(lib.cloudsc_state_sync(g.h))
            df.copy_from(sf, ["plude"])
            hip.hipEventRecord(e0, None)
            ca.check(lib.cloudsc_gpu_run(0, None, prec, variant, args.ngptot, args.nproma, ds.klev, C.byref(df.f),
                                         ws))
            hip.hipEventRecord(e1, None)
            hip.hipEventSynchronize(e1)
            t = C.c_float()
            hip.hipEventElapsedTime(C.byref(t), e0, e1)
            if i >= 5:
                ms.append(t.value)
        ca.check(lib.cloudsc_gpu_check(0, None, variant, ws))
    finally:
        for e in (e0, e1):
            if e.value:
                hip.hipEventDestroy(e)
        if ws.value:
            hip.hipFree(ws)
        rep = df.report.to_dict()
        df.close()
    return {"kernel_ms_median": round(float(np.median(ms)), 4), "kernel_ms_min": round(float(np.min(ms)), 4),
            "launches": len(ms), "placement": rep,
            "method": "cloudsc_fields_alloc (outputs placed by the read+write memory-pattern search) + cloudsc_gpu_run, the "
                      "reference CUDA driver's allocate / copy in / launch shape (cloudsc_driver.cu:276-416); "
                      "HIP events on the null stream around each launch (the KSEG prepare kernel included)"}


def energy_window(g, variant, cp, pw_file, seconds, ncols, np):
    """Board power while the kernel runs back to back for `seconds` (after the
    timed region, untimed): mean W over the window and the energy per column =
    mean W x time per launch / columns.  The sensor averages over ~1-10 ms,
    longer than one 1.6 ms launch, so the window is long; the timed region's
    own mean W is reported beside it."""
    if not pw_file:
        return {"board_w": None, "energy_uj_per_column": None, "source": "no hwmon power file for this device"}
    s = cp.PowerSampler(pw_file)
    s.start()
    t0, span, n = time.perf_counter(), 0.0, 0
    while time.perf_counter() - t0 < seconds:
        span += g.run_span(variant, 50)
        n += 50
    g.sync()
    s.stop()
    w = s.mean_w()
    k = span / n
    return {"board_w": round(w, 1) if w else None,
            "energy_uj_per_column": round(w * k * 1e-3 / ncols * 1e6, 3) if w else None,
            "kernel_ms": round(k, 4), "launches": n, "samples": len(s.samples),
            "seconds": round(time.perf_counter() - t0, 2), "source": pw_file,
            "method": "hwmon board power sampled every 10 ms while the kernel ran back to back after the timed "
                      "region (plain launches, timed 50 at a time); energy per column = mean W x time per launch / "
                      "columns (the reference reads energy beside its timings: EC_PMON, "
                      "src/common/module/ec_pmon_mod.F90)"}


def main():
    args = parse()
    import numpy as np
    import cloudsc_amd as ca
    import cloudsc_dist as cd
    import cloudsc_power as cp

    topo = cd.topology_from_env()
    ctl = cd.Control(topo)               # gloo: barrier + max-over-ranks only
    world, rank = topo.world, topo.rank
    col_offset, ncols = cd.shard(rank, args.ngptot)

    prec = ca.FP64 if args.precision == "fp64" else ca.FP32
    variant = {"kseg": ca.VARIANT_KSEG, "kcache": ca.VARIANT_KCACHE, "scc": ca.VARIANT_SCC,
               "scc-private": ca.VARIANT_SCC_PRIVATE}[args.variant]
    kind = variant
    if args.fp32_exact_libm:
        variant |= ca.FP32_EXACT_LIBM
    ds = ca.load_dataset()
    # one GPU per local rank (ranks beyond the device count share devices, e.g.
    # a 2-rank rehearsal on a 1-GPU box)
    device = topo.local_rank % ca.device_count()
    g = ca.GpuState(ds, ncols, args.nproma, prec, device=device, col_offset=col_offset)
    # one launch timed alone, as the reference GPU driver times its single launch
    # (cloudsc_driver.cu:389-422), right after creation (whose placement search
    # has already run the kernel; the clock is not yet settled)
    first_step_ms = float(g.run(variant, 1)[0])
    # The achievable-HBM (STREAM copy) measurement runs first: ~0.1 s of heavy
    # GPU work, after which the shader clock has left its idle level.  The
    # kernel's time follows the clock (profiles/r02/clock_probe_kseg_fp64.json:
    # 1.95 ms at 1.85 GHz for the first dispatches of a cold device, 1.68 ms at
    # 2.3 GHz once ramped), so a cold start would otherwise bias the first steps.
    peak_meas = None
    if not args.no_hbm_peak:          # every rank warms its own device the same way
        peak_meas = ca.hbm_copy_gbps(device, 4 << 30, 10)

    prewarm = prewarm_until_stable(g, variant, args.warmup, np)
    g.sync()
    if kind == ca.VARIANT_KSEG:
        g.kseg_clock(reset=True)                # the clock counters cover the timed launches only
    pw_file = cp.power_file(device)
    sampler = cp.PowerSampler(pw_file)
    ctl.barrier()
    sampler.start()
    t0 = time.perf_counter()
    # one plain launch per step, the K launches bracketed by two events on the state's stream: a dispatch
    # that records its own events leaves ~5 us more between kernels (profiles/r05/launch_forms.txt)
    span_ms = g.run_span(variant, args.steps)
    g.sync()
    t1 = time.perf_counter()
    sampler.stop()
    ctl.barrier()
    wall = ctl.max(t1 - t0)
    k_avg_ms = ctl.max(span_ms / args.steps)
    sclk = g.kseg_clock() if kind == ca.VARIANT_KSEG else None
    # the launch-time distribution: the same K launches again, each recording its own events (untimed),
    # with that pass's own effective shader clock.  After the timed region the device idles for the host's
    # bookkeeping, and the first ~10-20 launches after such a pause ran up to 17 % slow (profiles/r06: 1.72,
    # 1.87, 1.94, ... 1.66 ms, the same shape in fp32): the pass is re-warmed by time first, like the timed
    # region, so its percentiles describe the steady launches (round 5's driver run: p90 1.86 ms)
    rewarm = prewarm_until_stable(g, variant, 0, np, floor=10)
    if kind == ca.VARIANT_KSEG:
        g.kseg_clock(reset=True)
    kernel_ms = g.run(variant, args.steps)
    sclk2 = g.kseg_clock() if kind == ca.VARIANT_KSEG else None
    energy = energy_window(g, variant, cp, pw_file, args.energy_seconds, ncols, np) if args.energy_seconds > 0 \
        else None
    # ranks sharing one device (a rehearsal with more ranks than GPUs) read the same board over overlapping
    # windows: its power is theirs together, so no per-column energy is claimed
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    sharing = sum(1 for r in range(local_world) if r % ca.device_count() == device)
    if energy is not None and sharing > 1:
        energy["energy_uj_per_column"] = None
        energy["shared_device_note"] = ("%d ranks run on device %d at once: the board's power is theirs together, "
                                        "no per-column energy" % (sharing, device))
    if energy is not None:
        # the timed region's own board power only from >= 20 samples (4 samples of a sensor
        # that averages over 1-10 ms meant nothing); 100 launches of 1.65 ms give ~17 at 10 ms
        n_tr = len(sampler.samples)
        energy["timed_region_samples"] = n_tr
        energy["timed_region_board_w"] = round(sampler.mean_w(), 1) if sampler.mean_w() and n_tr >= 20 else None
        if n_tr < 20:
            energy["timed_region_board_w_note"] = "not reported: %d samples < 20 (see board_w over the window)" % n_tr
    # every rank's own record, gathered to rank 0 (the reference's per-rank
    # timing table, src/common/module/timer_mod.F90:160-167)
    mine = {"rank": rank, "device": device, "local_rank": topo.local_rank, "ngptot": ncols,
            "col_offset": col_offset, "wall_s": round(t1 - t0, 6),
            "kernel_ms": round(span_ms / args.steps, 4), "kernel_ms_min": round(float(np.min(kernel_ms)), 4),
            "kernel_ms_median": round(float(np.median(kernel_ms)), 4),
            "stream_gbs": round(peak_meas, 1) if peak_meas else None,
            "sclk_ghz": round(sclk, 4) if sclk else None, "prewarm_steps": prewarm,
            "first_step_ms": round(first_step_ms, 4),
            "board_w": energy.get("board_w") if energy else None,
            "energy_uj_per_column": energy.get("energy_uj_per_column") if energy else None,
            "placement": g.placement_report()}
    per_rank = ctl.gather_records(mine)

    # validation of the last step against reference.h5 (device-side statistics, combined over ranks)
    stats = ctl.gather_stats(g.validate())
    worst = 0.0
    for (mn, mx, maxerr, errsum, refsum) in (st[:5] for st in stats):
        worst = max(worst, errsum / refsum if refsum > 0 else errsum)
    boundary = None
    if not args.no_boundary and world == 1 and kind == ca.VARIANT_KSEG:
        boundary = boundary_path(ca, g, ds, args, prec, variant, np)
    g.close()

    if rank != 0:
        ctl.close()
        return

    total_cols = args.ngptot * world
    ms_per_step = 1e3 * wall / args.steps
    value = total_cols * args.steps / wall
    bpc = BYTES_PER_COL[prec]
    achieved = bpc * args.ngptot / (k_avg_ms * 1e-3) / 1e9
    traffic, traffic_src = roofline_traffic(
        ca, args.traffic_json, "%s_%s_%d_%d" % (args.variant, args.precision, args.ngptot, args.nproma))
    line = {
        "metric": "grid-columns/sec at NGPTOT=163840 KLEV=137 fp64; achieved HBM GB/s vs peak",
        "value": round(value, 1),
        "unit": "columns/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if prec == ca.FP64 else "f32",
        "data": "reference 100-column IFS state (data/cloudsc100, from the reference's data/) "
                "expanded on the device with g % 100",
        "config": {"workload": "CLOUDSC %s, NGPTOT=%d per GPU, KLEV=%d, NPROMA=%d, %s" % (
            {ca.VARIANT_KSEG: "SCC-k-caching (persistent, level-segmented)",
             ca.VARIANT_KCACHE: "SCC-k-caching", ca.VARIANT_SCC: "SCC (HBM temporaries)",
             ca.VARIANT_SCC_PRIVATE: "SCC (per-thread private-array temporaries)"}[kind],
            args.ngptot, ds.klev, args.nproma, args.precision),
            "libm": "reference CPU build's exp/pow (glibc algorithms)" if prec == ca.FP64 or args.fp32_exact_libm
                    else "float-internal expf/powf (hardware exp2/log2, exact argument reduction)",
            "ngptot_per_gpu": args.ngptot, "ngptot_total": total_cols, "klev": ds.klev,
            "nproma": args.nproma, "variant": args.variant, "parallelism": "columns sharded, %d GPU(s)" % world},
        "prewarm_steps": prewarm,
        "first_step_ms": round(first_step_ms, 4),
        "first_step_method": "one launch timed alone right after state creation, as cloudsc_driver.cu:389-422 times "
                             "its single launch (the placement search has run the kernel, the clock has not settled)",
        "kernel_ms": round(k_avg_ms, 4),
        "kernel_ms_min": round(float(np.min(kernel_ms)), 4),
        "kernel_ms_median": round(float(np.median(kernel_ms)), 4),
        "kernel_ms_p10": round(float(np.percentile(kernel_ms, 10)), 4),
        "kernel_ms_p90": round(float(np.percentile(kernel_ms, 90)), 4),
        "kernel_ms_method": "the timed region's K launches between two HIP events on the state's stream, / K (the "
                            "~1 us dispatch boundaries included); max over ranks.  min/median/p10/p90: a second "
                            "pass of K launches after the timed region, each recording its own events (+5 us "
                            "between kernels, not in the timed region)",
        "second_pass": {"sclk_ghz": round(sclk2, 4) if sclk2 else None, "rewarm_steps": rewarm,
                        "kernel_ms_hist": launch_histogram(kernel_ms, np),
                        "kernel_ms_all": [round(float(x), 4) for x in kernel_ms],
                        "method": "the per-launch times behind kernel_ms_median/p10/p90 (order of launch) and that "
                                  "pass's own effective shader clock (cloudsc_state_kseg_clock reset before it), after "
                                  "untimed re-warm launches until two batch medians agree (rewarm_steps)"},
        "sclk_ghz": round(sclk, 4) if sclk else None,
        "sclk_method": "effective shader clock of the timed launches: each workgroup's s_memtime cycles over its "
                       "s_memrealtime ticks, summed in the KSEG workspace (cloudsc_state_kseg_clock)",
        "box": box_info() if rank == 0 else None,
        "placement": dict(per_rank[0]["placement"], how=(
            "output placement search at state creation (cloudsc_state_placement_report): the KSEG kernel on the "
            "state's own inputs timed (best of 2 after 1) over candidate placements -- 8 whole fresh output sets, "
            "one output field at a time, then 4 whole fresh input sets (the sets after the first shuffled, with "
            "spacers) -- a candidate kept when it is > 1 % faster; probe ms of the first and the kept placement, "
            "its wall time, probe launches and the most candidate bytes held at once; rank 0; outside the timed "
            "region")),
        "energy": energy,
        "per_rank": per_rank,
        "validation_worst_rel_l1": worst,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_column": bpc,
                     "algorithmic_bytes_per_launch": bpc * args.ngptot},
    }
    if traffic:   # the measured HBM bytes of one launch over this run's kernel time
        line["roofline"]["traffic_gbs"] = round(traffic / (k_avg_ms * 1e6), 1)
    if peak_meas:
        line["roofline"]["achievable_peak"] = {
            "value": round(peak_meas, 1), "unit": "GB/s",
            "method": "STREAM copy on this device in this run (cloudsc_hbm_copy_gbps: three pairs of 2 GiB "
                      "buffers, 8 / 16 / 64 KiB tiles per workgroup, non-temporal and cached, 10 launches of each "
                      "shape per pair, the best launch)"}
        line["roofline"]["frac_of_achievable"] = round(achieved / peak_meas, 4)
    # the same against MI355X_MICROARCH.md's measured float4 copy (a fixed figure, not this box's)
    line["roofline"]["guide_copy_peak"] = {"value": GUIDE_COPY_GBS, "unit": "GB/s",
                                           "source": "MI355X_MICROARCH.md:36 (float4 copy, measured)"}
    line["roofline"]["frac_of_guide_copy"] = round(achieved / GUIDE_COPY_GBS, 4)
    if not args.no_transfer and world == 1:
        line["pcie_inclusive"] = transfer_rate(ca, ds, args, prec, variant)
    if boundary is not None:
        line["boundary_path"] = boundary
    if not args.no_cpu_baseline and world == 1:
        nth = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(ca, ds, nth)
    print(json.dumps(line), flush=True)
    ctl.close()


if __name__ == "__main__":
    main()
