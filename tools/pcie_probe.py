#!/usr/bin/env python3
"""Host<->device copy bandwidth of this box (the bound of the host-buffer
pipeline, DESIGN.md §7 / SURVEY §8 f3): pinned host buffers, H2D alone, D2H
alone, and both directions at once on two streams.  One JSON line."""
import json
import time

import torch


def timed(fn, reps=5):
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    nbytes = 1 << 30
    h_in = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_in.fill_(1)
    d_in = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_out.fill_(2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        d_in.copy_(h_in, non_blocking=True)

    def d2h():
        h_out.copy_(d_out, non_blocking=True)

    def both():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    h2d(); d2h(); both()
    t_h2d, t_d2h, t_both = timed(h2d), timed(d2h), timed(both)
    print(json.dumps({"bytes_each_direction": nbytes,
                      "h2d_GBs": round(nbytes / t_h2d / 1e9, 1),
                      "d2h_GBs": round(nbytes / t_d2h / 1e9, 1),
                      "both_directions_GBs_total": round(2 * nbytes / t_both / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
