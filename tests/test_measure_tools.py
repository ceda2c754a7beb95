"""Host-side pieces of the round-5 measurements, without a GPU: the board-power
sampler of bench.py (cloudsc_power), the selection of the timed launches from a
rocprofv3 kernel trace (tools/timed_stats.py), the counter calibration's
analysis (tools/calib_counters.py), the argument checks of the new C entry
points that run before any device call, and the CLI's --place option."""
import csv
import ctypes as C
import json
import os
import subprocess
import sys

import pytest

import cloudsc_amd as ca
import cloudsc_power as cp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(REPO, "tools")
sys.path.insert(0, TOOLS)


def test_power_sampler_reads_microwatts(tmp_path):
    f = tmp_path / "power1_input"
    f.write_text("1350000000\n")                 # 1350 W in microwatts, as hwmon reports it
    s = cp.PowerSampler(str(f), period=0.001)
    s.start()
    import time
    time.sleep(0.02)
    s.stop()
    assert s.samples and abs(s.mean_w() - 1350.0) < 1e-9
    assert cp.PowerSampler(None).read_w() is None
    assert cp.PowerSampler(str(tmp_path / "missing")).read_w() is None


def test_power_file_without_a_device_is_none():
    # no HIP device in this container: no bus id, so no file (bench.py then reports None)
    assert cp.power_file(0) is None or os.path.exists(cp.power_file(0))


def test_timed_stats_selects_the_timed_launches(tmp_path):
    import timed_stats
    trace = tmp_path / "k_kernel_trace.csv"
    before, steps = 7, 5                          # placement launches 4 + first step 1 + prewarm 2
    rows = []
    t = 1000
    for i in range(before + steps + 3):           # 3 more after (the energy window)
        dur = 100 + (50 if before <= i < before + steps else 0)
        rows.append({"Kernel_Name": "void kseg_entry<double, 2, 3>", "Start_Timestamp": t, "End_Timestamp": t + dur})
        rows.append({"Kernel_Name": "kseg_prepare_kernel", "Start_Timestamp": t + 1, "End_Timestamp": t + 2})
        t += 1000
    with open(trace, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    bench = tmp_path / "bench.log"
    bench.write_text("noise\n" + json.dumps({"placement": {"launches": 4}, "prewarm_steps": 2, "steps": steps,
                                             "kernel_ms": 0.00015, "kernel_ms_median": 0.00015}) + "\n")
    sys.argv = ["timed_stats.py", str(trace), str(bench), str(tmp_path / "out")]
    timed_stats.main()
    d = [int(x) for x in open(tmp_path / "out_timed_durations.txt") if not x.startswith("#")]
    assert d == [150] * steps
    row = list(csv.DictReader(open(tmp_path / "out_timed_stats.csv")))[0]
    assert int(row["Calls"]) == steps and float(row["AverageNs"]) == 150.0


def test_calibration_analysis(tmp_path):
    import calib_counters
    gib, reps = 4.0, 3
    nbytes = gib * (1 << 30)
    for counter, d in (("FETCH_SIZE", "f"), ("WRITE_SIZE", "w")):
        os.makedirs(tmp_path / d)
        with open(tmp_path / d / "calib_counter_collection.csv", "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            did = 0
            for mode in ("read", "write"):
                for width in (4, 8, 16):
                    for _ in range(reps):
                        did += 1
                        if counter == "FETCH_SIZE":
                            kb = nbytes / 2 / 1024 if mode == "read" else 10.0
                        else:
                            kb = nbytes / 1024 if mode == "write" else 0.0
                        w.writerow({"Dispatch_Id": did, "Kernel_Name": "stream_probe<%d>" % width,
                                    "Counter_Name": counter, "Counter_Value": kb})
    out = tmp_path / "traffic.json"
    calib_counters.analyse(str(tmp_path / "f"), str(tmp_path / "w"), str(out), gib, reps)
    res = json.load(open(out))["calibration"]["results"]
    for width in (4, 8, 16):
        assert res["read_%dB_per_lane" % width]["FETCH_SIZE"]["bytes_per_counter_byte"] == 2.0
        assert res["write_%dB_per_lane" % width]["WRITE_SIZE"]["bytes_per_counter_byte"] == 1.0


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(ca.LIB_PATH):
        pytest.skip("libcloudsc_amd.so not built")
    return ca.gpu_lib()


def test_new_entry_points_check_arguments_first(lib):
    """Checks that run before any device call (no GPU here)."""
    f, r = ca.Fields(), ca.Placement()
    assert lib.cloudsc_fields_alloc(0, ca.FP64, 1000, 128, 137, 4, C.byref(f), C.byref(r)) == ca.EINVAL
    assert lib.cloudsc_fields_alloc(0, ca.FP64, 1000, 128, 137, 0, None, C.byref(r)) == ca.EINVAL
    assert lib.cloudsc_fields_free(0, None) == ca.EINVAL
    assert lib.cloudsc_set_placement_search(9) == ca.EINVAL
    assert lib.cloudsc_set_placement_search(-1) == 0
    live, bad, nb = C.c_int(), C.c_int(), C.c_longlong()
    lib.cloudsc_debug_canary_check.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
    assert lib.cloudsc_debug_canary_check(C.byref(live), C.byref(bad), C.byref(nb)) == ca.EINVAL  # product build
    ms = C.c_double()
    lib.cloudsc_debug_stream_probe.argtypes = [C.c_int, C.c_int, C.c_int, C.c_longlong, C.c_int,
                                               C.POINTER(C.c_double)]
    assert lib.cloudsc_debug_stream_probe(0, 0, 12, 1 << 30, 1, C.byref(ms)) == ca.EINVAL
    assert lib.cloudsc_debug_stream_probe(0, 2, 8, 1 << 30, 1, C.byref(ms)) == ca.EINVAL
    lib.cloudsc_debug_kernel_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong]
    assert lib.cloudsc_debug_kernel_copy(None, None, 16) == ca.EINVAL
    assert lib.cloudsc_debug_memory_probe(0, ca.FP64, 1000, 128, 137, None, 0, 1, C.byref(C.c_float())) == ca.EINVAL
    lib.cloudsc_debug_memory_probe_layout.argtypes = [C.c_int] * 5 + [C.c_void_p, C.c_int, C.c_int,
                                                                      C.POINTER(C.c_longlong), C.POINTER(C.c_float)]
    assert lib.cloudsc_debug_memory_probe_layout(0, ca.FP64, 1000, 128, 137, None, 1, 1, None,
                                                 C.byref(C.c_float())) == ca.EINVAL
    neg = (C.c_longlong * 6)(0, 0, 0, -1, 0, 0)
    assert lib.cloudsc_debug_memory_probe_layout(0, ca.FP64, 1000, 128, 137, C.byref(f), 1, 1, neg,
                                                 C.byref(C.c_float())) == ca.EINVAL
    assert C.sizeof(ca.Placement) == 48   # cloudsc_placement_t with transient_budget_bytes (round 6)


def test_cli_place_option():
    dwarf = os.path.join(REPO, "dwarf-p-cloudsc_amd", "dwarf-cloudsc-amd")
    if not os.path.exists(dwarf):
        pytest.skip("dwarf-cloudsc-amd not built")
    bad = subprocess.run([dwarf, "1", "100", "4", "--place", "maybe"], capture_output=True, text=True)
    assert bad.returncode != 0 and "bad --place" in bad.stderr
    usage = subprocess.run([dwarf, "--help"], capture_output=True, text=True)
    assert "--place on|off|auto" in usage.stderr
    ok = subprocess.run([dwarf, "1", "200", "16", "--variant", "cpu", "--place", "off"], capture_output=True,
                        text=True, timeout=120)
    assert ok.returncode == 0 and "VALIDATION: PASSED" in ok.stdout, ok.stdout[-1500:] + ok.stderr


def test_cli_energy_option():
    dwarf = os.path.join(REPO, "dwarf-p-cloudsc_amd", "dwarf-cloudsc-amd")
    if not os.path.exists(dwarf):
        pytest.skip("dwarf-cloudsc-amd not built")
    for v in ("-1", "x", "1000"):
        bad = subprocess.run([dwarf, "1", "100", "4", "--energy", v], capture_output=True, text=True)
        assert bad.returncode != 0 and "bad --energy" in bad.stderr
    usage = subprocess.run([dwarf, "--help"], capture_output=True, text=True)
    assert "--energy S" in usage.stderr
    ok = subprocess.run([dwarf, "1", "200", "16", "--variant", "cpu", "--energy", "0.1"], capture_output=True,
                        text=True, timeout=120)
    assert ok.returncode == 0 and "VALIDATION: PASSED" in ok.stdout, ok.stdout[-1500:] + ok.stderr
    assert " ENERGY: n/a (host variant" in ok.stdout
