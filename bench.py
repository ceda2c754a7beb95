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
wall time.  The kernel alone is also timed with HIP events recorded on the
launch stream (roofline.achieved uses that kernel time).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))

BYTES_PER_COL = {8: 56036, 4: 28020}     # SURVEY.md §8d algorithmic bytes per column
HBM_PEAK_GBS = 8000.0                    # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)    # 0.2 s of kernels: a stable mean
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--ngptot", type=int, default=163840, help="columns per GPU")
    p.add_argument("--nproma", type=int, default=64,
                   help="NPROMA (block = workgroup); 64 is the measured best for the persistent kernel "
                        "(profiles/r01/nproma_sweep_all_variants.jsonl)")
    p.add_argument("--precision", choices=["fp64", "fp32"], default="fp64")
    p.add_argument("--variant", choices=["kseg", "kcache", "scc"], default=None,
                   help="default: kseg for fp64 (2 waves/SIMD leave a tail the persistent kernel removes), "
                        "kcache for fp32 (3-4 waves/SIMD, no tail)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--transfer", action="store_true",
                   help="also time the host-buffer path (H2D -> kernel -> D2H, chunked over streams): "
                        "reported as pcie_inclusive, never as value")
    p.add_argument("--transfer-steps", type=int, default=3)
    p.add_argument("--cpu-sample", type=int, default=65536, help="columns in the CPU baseline sample")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_latest.json"),
                   help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    a = p.parse_args()
    if a.variant is None:
        a.variant = "kseg" if a.precision == "fp64" else "kcache"
    return a


def cpu_baseline(ds, ncols, nproma=32):
    """Reference C kernel (oracle/_ref, compiled from the reference sources) when
    present, else the oracle restatement; OpenMP over NPROMA blocks on the host
    cores (cloudsc_driver.c:183-217).  Returns the cpu_baseline object."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    kind = "reference" if oracle.ref_available() else "port"
    best = None
    for _ in range(2):
        if kind == "reference":
            _, secs = oracle.run_ref(ds, ncols, nproma, nthreads=nthreads)
        else:
            _, secs = oracle.run_oracle(ds, ncols, nproma, nthreads=nthreads)
        best = secs if best is None else min(best, secs)
    return {"value": ncols / best, "unit": "columns/s", "cores": nthreads, "kind": kind,
            "sample": "%d columns of the same fp64 workload (g %% 100 expansion, KLEV=137), NPROMA=%d, "
                      "%d OpenMP threads, best of 2 block loops (%s)" % (
                          ncols, nproma, nthreads,
                          "src/cloudsc_c/cloudsc/cloudsc_c.c" if kind == "reference" else "oracle/cloudsc_oracle.c")}


def transfer_rate(ca, ds, args, prec, variant, chunk_blocks=32, nstreams=4):
    """Host-resident block-layout arrays (pinned in place), per chunk H2D ->
    kernel -> D2H overlapped on streams: the reference GPU drivers' TOTAL
    semantics (cloudsc_driver.cu:344-456).  plude is restored on the host
    between steps, outside the timed pipeline."""
    hp = ca.HostPipeline(ds, args.ngptot, args.nproma, prec, chunk_blocks=chunk_blocks, nstreams=nstreams)
    try:
        hp.run(variant)
        ms = [hp.run(variant) for _ in range(args.transfer_steps)]
    finally:
        hp.close()
    t = sum(ms) / len(ms)
    return {"value": round(args.ngptot / (t * 1e-3), 1), "unit": "columns/s", "ms_per_step": round(t, 3),
            "chunk_blocks": chunk_blocks, "nstreams": nstreams,
            "bytes_per_step": BYTES_PER_COL[prec] * args.ngptot,
            "note": "host-buffer path incl. PCIe H2D/D2H; not the headline value"}


def main():
    args = parse()
    import numpy as np
    import cloudsc_amd as ca
    import cloudsc_dist as cd

    topo = cd.topology_from_env()
    ctl = cd.Control(topo)               # gloo: barrier + max-over-ranks only
    world, rank = topo.world, topo.rank
    col_offset, ncols = cd.shard(rank, args.ngptot)

    prec = ca.FP64 if args.precision == "fp64" else ca.FP32
    variant = {"kseg": ca.VARIANT_KSEG, "kcache": ca.VARIANT_KCACHE, "scc": ca.VARIANT_SCC}[args.variant]
    ds = ca.load_dataset()
    # one GPU per local rank (ranks beyond the device count share devices, e.g.
    # a 2-rank rehearsal on a 1-GPU box)
    device = topo.local_rank % ca.device_count()
    g = ca.GpuState(ds, ncols, args.nproma, prec, device=device, col_offset=col_offset)

    if args.warmup > 0:
        g.run(variant, args.warmup)
    g.sync()
    ctl.barrier()
    t0 = time.perf_counter()
    kernel_ms = g.run(variant, args.steps)      # one launch per step; events around each launch
    g.sync()
    t1 = time.perf_counter()
    ctl.barrier()
    wall = ctl.max(t1 - t0)
    k_avg_ms = ctl.max(float(np.mean(kernel_ms)))

    # validation of the last step against reference.h5 (device-side statistics, combined over ranks)
    stats = ctl.gather_stats(g.validate())
    worst = 0.0
    for (mn, mx, maxerr, errsum, refsum) in stats:
        worst = max(worst, errsum / refsum if refsum > 0 else errsum)
    g.close()

    if rank != 0:
        ctl.close()
        return

    total_cols = args.ngptot * world
    ms_per_step = 1e3 * wall / args.steps
    value = total_cols * args.steps / wall
    bpc = BYTES_PER_COL[prec]
    achieved = bpc * args.ngptot / (k_avg_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            key = "%s_%s_%d_%d" % (args.variant, args.precision, args.ngptot, args.nproma)
            if key in tj:
                traffic = tj[key]["hbm_bytes_per_launch"]
        except Exception:
            traffic = None
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
        "data": "reference 100-column IFS state (tests/golden/cloudsc100, from the reference's data/) "
                "expanded on the device with g % 100",
        "config": {"workload": "CLOUDSC %s, NGPTOT=%d per GPU, KLEV=%d, NPROMA=%d, %s" % (
            {ca.VARIANT_KSEG: "SCC-k-caching (persistent, level-segmented)",
             ca.VARIANT_KCACHE: "SCC-k-caching", ca.VARIANT_SCC: "SCC (HBM temporaries)"}[variant],
            args.ngptot, ds.klev, args.nproma, args.precision),
            "ngptot_per_gpu": args.ngptot, "ngptot_total": total_cols, "klev": ds.klev,
            "nproma": args.nproma, "variant": args.variant, "parallelism": "columns sharded, %d GPU(s)" % world},
        "kernel_ms": round(k_avg_ms, 4),
        "kernel_ms_min": round(float(np.min(kernel_ms)), 4),
        "validation_worst_rel_l1": worst,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "algorithmic_bytes_per_column": bpc},
    }
    if args.transfer and world == 1:
        line["pcie_inclusive"] = transfer_rate(ca, ds, args, prec, variant)
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(ds, min(args.cpu_sample, args.ngptot))
    print(json.dumps(line), flush=True)
    ctl.close()


if __name__ == "__main__":
    main()
