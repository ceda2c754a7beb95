#!/usr/bin/env python3
"""A few launches of the library's STREAM copy (cloudsc_hbm_copy_gbps) for
counter passes beside the kernel's (tools/pmc_tlb.sh, KREGEX=copy)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402

print("STREAM copy %.1f GB/s" % ca.hbm_copy_gbps(0, 4 << 30, 3))
