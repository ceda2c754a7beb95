"""Debug: where do GPU fp32 and the fp32 oracle differ (sign of zero)?"""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd")); sys.path.insert(0, os.path.join(REPO, "oracle"))
import cloudsc_amd as ca, oracle
ds = ca.load_dataset()
for var in (ca.VARIANT_KCACHE, ca.VARIANT_KSEG, ca.VARIANT_SCC):
    g = ca.GpuState(ds, 100, 100, ca.FP32)
    g.run(var, 1); out = g.outputs(); g.close()
    st, _ = oracle.run_oracle(ds, 100, 100, ca.FP32)
    ref = ca.state_outputs_to_template(st.arrays, 100)
    for _, k in ca.VALIDATED:
        a = out[k].astype(np.float32).view(np.uint32); r = ref[k].astype(np.float32).view(np.uint32)
        d = np.argwhere(a != r)
        if len(d):
            i = tuple(d[0])
            print(var, k, len(d), "first", i, hex(int(a[i])), hex(int(r[i])), "levels", sorted(set(int(x[-2]) for x in d))[:20])
