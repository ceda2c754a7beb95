"""Child of tests/test_dist.py::test_gloo_connect_leaves_stdout_to_rank0: a
two-rank group connects through cloudsc_dist.Control, then rank 0 alone
prints one line (as bench.py prints its JSON result)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dwarf-p-cloudsc_amd"))
import cloudsc_dist as cd  # noqa: E402

topo = cd.topology_from_env()
ctl = cd.Control(topo)
ctl.barrier()
if topo.rank == 0:
    print('{"rank0": true}', flush=True)
ctl.barrier()
ctl.close()
