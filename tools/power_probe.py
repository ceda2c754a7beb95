#!/usr/bin/env python3
"""Board power and energy per column of the KSEG kernel (VERDICT r03 weak #4:
the fp64 "power-bound" reading needs a power sample, not only clocks).

For each library given (e.g. the full kernel and the memory-only ablation of
tools/ablation.sh), one device state runs the kernel back to back for about
`--seconds` while a sampler thread reads the board's power: the hwmon
power1_average / power1_input of the GPU (sysfs, microwatts) when readable, else
`amd-smi metric -p --json`.  Reported per library: mean / max power over the
busy window, kernel time, the effective shader clock of the launches
(cloudsc_state_kseg_clock) and the energy per column (mean power x kernel time /
columns).  One JSON line per library.
usage: power_probe.py [--seconds 8] [--precision fp64] lib.so ..."""
import argparse
import glob
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402


def hwmon_power_files():
    out = []
    for d in sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*")):
        for name in ("power1_average", "power1_input"):
            f = os.path.join(d, name)
            try:
                with open(f) as fh:
                    int(fh.read().strip())
                out.append(f)
                break
            except (OSError, ValueError):
                continue
    return out


def read_smi_watts():
    r = subprocess.run(["amd-smi", "metric", "-p", "--json"], capture_output=True, text=True, timeout=10)
    data = json.loads(r.stdout)
    gpus = data if isinstance(data, list) else data.get("gpu_data", [data])
    vals = []
    for g in gpus:
        p = g.get("power", {})
        for key in ("socket_power", "average_socket_power", "current_socket_power"):
            v = p.get(key)
            if isinstance(v, dict):
                v = v.get("value")
            if isinstance(v, (int, float)):
                vals.append(float(v))
                break
    return vals


class Sampler(threading.Thread):
    def __init__(self, period=0.05):
        super().__init__(daemon=True)
        self.files = hwmon_power_files()
        self.source = "hwmon " + ",".join(self.files) if self.files else "amd-smi metric -p"
        self.period = period if self.files else 0.25
        self.samples = []
        self.stop_ev = threading.Event()

    def read(self):
        if self.files:   # the card with the highest reading is the busy one (one GPU per box)
            vals = []
            for f in self.files:
                with open(f) as fh:
                    vals.append(int(fh.read().strip()) * 1e-6)
            return max(vals)
        v = read_smi_watts()
        return max(v) if v else None

    def run(self):
        while not self.stop_ev.is_set():
            try:
                w = self.read()
                if w is not None:
                    self.samples.append((time.perf_counter(), w))
            except Exception as e:   # keep sampling; report what failed once
                self.samples.append((time.perf_counter(), None))
                self.error = repr(e)
            time.sleep(self.period)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=8.0)
    p.add_argument("--precision", default="fp64")
    p.add_argument("--ngptot", type=int, default=163840)
    p.add_argument("libs", nargs="+")
    a = p.parse_args()
    prec = ca.FP64 if a.precision == "fp64" else ca.FP32
    ds = ca.load_dataset()
    idle = Sampler()
    idle.start()
    time.sleep(1.0)
    idle.stop_ev.set()
    idle.join()
    idle_w = [w for _, w in idle.samples if w is not None]
    print(json.dumps({"idle_watts": round(sum(idle_w) / len(idle_w), 1) if idle_w else None,
                      "source": idle.source}), flush=True)
    for path in a.libs:
        ca._lib = None
        ca.gpu_lib(os.path.realpath(path))
        g = ca.GpuState(ds, a.ngptot, 64, prec)
        try:
            g.run(ca.VARIANT_KSEG, 30)            # clock ramp
            g.kseg_clock(reset=True)
            s = Sampler()
            s.start()
            t0 = time.perf_counter()
            ms = []
            while time.perf_counter() - t0 < a.seconds:
                ms.extend(g.run(ca.VARIANT_KSEG, 50).tolist())
            t1 = time.perf_counter()
            s.stop_ev.set()
            s.join()
            ghz = g.kseg_clock()
        finally:
            g.close()
        busy = [w for t, w in s.samples if w is not None and t0 + 0.5 <= t <= t1]
        k = sorted(ms)[len(ms) // 2]
        mean_w = sum(busy) / len(busy) if busy else None
        print(json.dumps({"lib": os.path.basename(path), "kernel_ms_median": round(k, 4), "launches": len(ms),
                          "sclk_ghz": round(ghz, 3), "power_w_mean": round(mean_w, 1) if mean_w else None,
                          "power_w_max": round(max(busy), 1) if busy else None, "samples": len(busy),
                          "energy_uj_per_column": round(mean_w * k * 1e-3 / a.ngptot * 1e6, 4) if mean_w else None,
                          "source": s.source, "error": getattr(s, "error", None)}), flush=True)


if __name__ == "__main__":
    main()
