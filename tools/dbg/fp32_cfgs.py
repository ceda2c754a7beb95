"""Debug: fp32 KCACHE bit-identity vs the fp32 oracle per kernel configuration."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd")); sys.path.insert(0, os.path.join(REPO, "oracle"))
import cloudsc_amd as ca, oracle
ds = ca.load_dataset()
st, _ = oracle.run_oracle(ds, 100, 100, ca.FP32)
ref = ca.state_outputs_to_template(st.arrays, 100)
for cfg in sys.argv[1].split(","):
    os.environ["CLOUDSC_KCACHE_CFG"] = cfg
    for var in (ca.VARIANT_KCACHE, ca.VARIANT_KSEG):
        g = ca.GpuState(ds, 100, 100, ca.FP32)
        g.run(var, 1); out = g.outputs(); g.close()
        bad = []
        for _, k in ca.VALIDATED:
            a = out[k].astype(np.float32).view(np.uint32); r = ref[k].astype(np.float32).view(np.uint32)
            n = int(np.count_nonzero(a != r))
            if n: bad.append((k, n))
        print("cfg", cfg, "variant", var, bad, flush=True)
