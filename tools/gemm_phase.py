"""Per-workgroup phase timing of one BN-backward dgrad GEMM launch inside the config-2 step.

Needs the timing build: bash tools/build_ab.sh ts -DURED_GEMM_TIMING=1 -DURED_TS_M=32768
-DURED_TS_N=1024 -DURED_TS_K=512, then URED_LIB=build_ab/ts.so python tools/gemm_phase.py.
Runs the bench (short), then reads the last recorded launch of that shape: per workgroup the
real-time clock (100 MHz) at start, first K-step ready, K-loop end, epilogue end, and where it ran.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sys.argv = ["bench.py", "--no-cpu-baseline", "--no-all-slots-rate", "--no-k16-rate", "--no-extras",
                "--steps", "5", "--warmup", "2"]
    import bench
    bench.main()
    lib = ctypes.CDLL(os.environ["URED_LIB"])
    n = 8192
    buf = (ctypes.c_ulonglong * (n * 16))()
    assert lib.ured_debug_gemm_ts(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 16)
    bid = np.nonzero(a[:, 7] == 1)[0]          # slot = blockIdx.x
    a = a[a[:, 7] == 1]
    if len(a) == 0:
        print("no workgroup recorded (shape not launched?)")
        return
    t = a[:, :4].astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) * 10e-3          # us (100 MHz)
    hw = a[:, 4].astype(np.int64)
    xcc = a[:, 5].astype(np.int64) & 0xF
    cu = (xcc << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
    ready, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    e = (a[:, 8:12].astype(np.int64) - t0) * 10e-3
    if (a[:, 8] > 0).all():     # the full-tile BN-backward epilogue's marks
        for name, v in (("epi: Yp + params landed", e[:, 0] - t[:, 2]), ("epi: compute + G stores", e[:, 1] - e[:, 0]),
                        ("epi: column sums via LDS", e[:, 2] - e[:, 1]), ("epi: partials written", e[:, 3] - e[:, 2]),
                        ("epi: store drain", t[:, 3] - e[:, 3])):
            print(f"  {name:26s} mean {v.mean():7.2f}  p10 {np.percentile(v, 10):7.2f}  "
                  f"p50 {np.percentile(v, 50):7.2f}  p90 {np.percentile(v, 90):7.2f} us")
    span = t[:, 3].max()
    print(f"workgroups {len(a)}  CUs {len(np.unique(cu))}  launch span {span:.1f} us")
    for name, v in (("start->first step ready", ready), ("K-loop", loop), ("epilogue", epi),
                    ("whole tile", t[:, 3] - t[:, 0])):
        print(f"  {name:26s} mean {v.mean():7.2f}  p10 {np.percentile(v, 10):7.2f}  "
              f"p50 {np.percentile(v, 50):7.2f}  p90 {np.percentile(v, 90):7.2f} us")
    # per CU: how many tiles, and the time no workgroup of this launch was resident on it
    idle, ntile, conc = [], [], []
    for c in np.unique(cu):
        s = t[cu == c]
        ntile.append(len(s))
        ev = sorted([(x, 1) for x in s[:, 0]] + [(x, -1) for x in s[:, 3]])
        live, last, busy, c2 = 0, 0.0, 0.0, 0.0
        for x, d in ev:
            if live > 0:
                busy += x - last
            if live >= 2:
                c2 += x - last
            live += d
            last = x
        idle.append(span - busy)
        conc.append(c2 / max(busy, 1e-9))
    print(f"  tiles per CU: min {min(ntile)} max {max(ntile)}; CU idle within the launch: mean "
          f"{np.mean(idle):.1f} us, max {np.max(idle):.1f}; time with 2 resident: {np.mean(conc):.2f}")
    # placement: which block indices share a CU in the first round
    first = t[:, 0] < 1.0
    pairs = {}
    for b, c in zip(bid[first], cu[first]):
        pairs.setdefault(int(c), []).append(int(b))
    ks = sorted(pairs)[:12]
    print("  first-round blocks per CU (first 12 CUs):", [sorted(pairs[k]) for k in ks])
    sec = [sorted(v)[1] - sorted(v)[0] for v in pairs.values() if len(v) == 2]
    if sec:
        print("  index distance between a CU's two first-round blocks: min %d max %d, most common %s" % (
            min(sec), max(sec), np.bincount(np.array(sec) - min(sec)).argmax() + min(sec)))
    # start waves: how synchronous are the co-resident pairs
    order = np.argsort(t[:, 0])
    print("  first 8 starts (us):", np.round(t[order[:8], 0], 2).tolist())
    print("  tile start histogram (10 us bins):", np.histogram(t[:, 0], bins=np.arange(0, span + 10, 10))[0].tolist())
    print("  tile end histogram (10 us bins):  ", np.histogram(t[:, 3], bins=np.arange(0, span + 10, 10))[0].tolist())


if __name__ == "__main__":
    main()
