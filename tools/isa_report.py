"""Per-kernel ISA summary of the gemm2 variants (device asm from hipcc -S).

  python tools/isa_report.py mlp.s [kernel-substring]
For each kernel: VGPR/SGPR counts, spills, and the loop body that holds the MFMAs (the
basic-block loop containing the first v_mfma): instruction mix and every s_waitcnt in it.
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S*gemm2_kernel\S*):", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        yield m.group(1), text[start:end]


def meta(text, name):
    i = text.find(".name:           " + name)
    blk = text[i:i + 3000]
    g = lambda k: (re.search(k + r":\s+(\d+)", blk) or [None, "?"])[1]
    return g(r"\.vgpr_count"), g(r"\.sgpr_count"), g(r"\.vgpr_spill_count"), g(r"\.sgpr_spill_count")


def main(path, sub=""):
    text = open(path).read()
    for name, body in kernels(text):
        if sub not in name:
            continue
        lines = [l.strip() for l in body.splitlines() if l.strip() and not l.strip().startswith(";")]
        first = next((i for i, l in enumerate(lines) if l.startswith("v_mfma")), None)
        if first is None:
            continue
        # loop = from the last label before the first MFMA whose name is branched to after it
        labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r"(\.LBB\w+):", l)] if m}
        # the smallest backward-branch loop that encloses >= 64 MFMAs
        loop = None
        for i, l in enumerate(lines):
            m = re.match(r"s_c?branch\w*\s+(\.LBB\w+)", l)
            if not m or m.group(1) not in labels:
                continue
            t = labels[m.group(1)]
            if t < i and sum(x.startswith("v_mfma") for x in lines[t:i + 1]) >= 64:
                if loop is None or i - t < loop[1] - loop[0]:
                    loop = (t, i)
        v, s_, vs, ss = meta(text, name)
        short = re.sub(r"_ZN12_GLOBAL__N_112|EEEv12UredGemmDesc", "", name)
        print(f"{short}: vgpr {v} sgpr {s_} spills v{vs}/s{ss}")
        if loop:
            body_l = lines[loop[0]:loop[1] + 1]
            mf = sum(l.startswith("v_mfma") for l in body_l)
            waits = [l for l in body_l if l.startswith("s_waitcnt")]
            nvm = sum("vmcnt" in l for l in body_l if l.startswith("s_waitcnt"))
            print(f"   loop {len(body_l)} instr, {mf} mfma, {sum(l.startswith('ds_read') for l in body_l)} ds_read, "
                  f"{sum('buffer_load' in l for l in body_l)} dma, {sum(l.startswith('v_readlane') or l.startswith('v_writelane') for l in body_l)} lane-spill, "
                  f"{sum(l.startswith('s_barrier') for l in body_l)} barrier, {nvm} vmcnt waits (1 expected: the pre-barrier asm)")


if __name__ == "__main__":
    main(*sys.argv[1:3])
