EDITS = [("cloudsc_gpu.hip",
"""int kseg_nsub(int nproma) { return (nproma + 63) / 64; }
int kseg_wg(int nproma) { return nproma < 64 ? nproma : 64; }""",
"""int kseg_nsub(int nproma) { return nproma <= 256 ? 1 : (nproma + 63) / 64; }
int kseg_wg(int nproma) { return nproma <= 256 ? nproma : 64; }""")]
EDITS.append(("cloudsc_gpu.hip", "static std::atomic<int> cache[65];", "static std::atomic<int> cache[257];"))
