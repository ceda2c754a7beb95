import os, sys, time
sys.path.insert(0, 'dwarf-p-cloudsc_amd')
import numpy as np
import cloudsc_amd as ca
ds = ca.load_dataset()
mode = sys.argv[1]
os.environ['CLOUDSC_KCACHE_CFG'] = sys.argv[2]
if len(sys.argv) > 3: os.environ['CLOUDSC_KSEG_NSEG'] = sys.argv[3]
var = {'kseg': ca.VARIANT_KSEG, 'kcache': ca.VARIANT_KCACHE}[mode]
ref = None
g = ca.GpuState(ds, 1000, 128)
t = time.time()
try:
    ms = g.run(var, 1)
    print(mode, sys.argv[2:], 'ms', ms, 'wall', time.time() - t, flush=True)
    out = g.outputs()
finally:
    g.close()
os.environ['CLOUDSC_KCACHE_CFG'] = '20'
g = ca.GpuState(ds, 1000, 128); g.run(ca.VARIANT_KCACHE, 1); ref = g.outputs(); g.close()
bad = [k for _, k in ca.VALIDATED if not np.array_equal(out[k], ref[k])]
print('differ:', bad, flush=True)
