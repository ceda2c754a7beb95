"""bench.py's host-side helpers, without a GPU: the roofline's measured traffic
is taken only from a PMC record of the current kernel sources (a stale,
missing or unreadable record gives null with the reason), and the algorithmic
bytes per column are SURVEY.md §8(d)'s."""
import json
import os
import sys

import cloudsc_amd as ca

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

KEY = "kseg_fp64_163840_64"


def test_traffic_taken_only_from_the_current_kernel_sources(tmp_path):
    f = tmp_path / "traffic.json"
    f.write_text(json.dumps({KEY: {"kernel_source_hash": ca.kernel_source_hash(), "hbm_bytes_per_launch": 9.25e9}}))
    v, why = bench.roofline_traffic(ca, str(f), KEY)
    assert v == 9.25e9 and ca.kernel_source_hash() in why
    f.write_text(json.dumps({KEY: {"kernel_source_hash": "0123456789abcdef", "hbm_bytes_per_launch": 9.25e9}}))
    v, why = bench.roofline_traffic(ca, str(f), KEY)
    assert v is None and "stale" in why
    v, why = bench.roofline_traffic(ca, str(f), "kseg_fp32_163840_64")
    assert v is None and "no PMC measurement" in why
    f.write_text("{not json")
    v, why = bench.roofline_traffic(ca, str(f), KEY)
    assert v is None and "unreadable" in why
    v, why = bench.roofline_traffic(ca, str(tmp_path / "absent.json"), KEY)
    assert v is None and "no PMC measurement" in why


def test_kernel_source_hash_covers_the_kernel_sources():
    h = ca.kernel_source_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    for name in ca.KERNEL_SOURCES:
        assert os.path.exists(os.path.join(REPO, "dwarf-p-cloudsc_amd", "csrc", name)), name


def test_algorithmic_bytes_per_column():
    # 3701 values read (+ the 4-byte ktype) and 3303 written per column
    assert bench.BYTES_PER_COL[8] == (3701 + 3303) * 8 + 4
    assert bench.BYTES_PER_COL[4] == (3701 + 3303) * 4 + 4
    assert bench.IN_BYTES_PER_COL[8] + 3303 * 8 == bench.BYTES_PER_COL[8]


def test_launch_histogram_counts_every_launch():
    import numpy as np
    ms = [1.650, 1.6551, 1.659, 1.701, 1.862]
    h = bench.launch_histogram(ms, np)
    assert h["width_us"] == 10.0 and h["lo_ms"] <= min(ms)
    assert sum(h["counts"]) == len(ms) and h["counts"][0] >= 1
    # the slowest launch falls in the last bin
    assert len(h["counts"]) == int((max(ms) - h["lo_ms"]) * 1e3 // 10.0) + 1


def test_host_cores_states_the_cpu_share():
    h = bench.host_cores()
    assert h["nproc"] == os.cpu_count() and h["nproc"] >= 1
    assert h["affinity_cpus"] is None or 1 <= h["affinity_cpus"] <= h["nproc"]
    assert h["sockets"] is None or h["sockets"] >= 1
