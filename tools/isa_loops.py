"""Dev tool: VALU / SALU / DS instructions per iteration of the block kernel's decode loops, from
the gfx950 ISA of dq_inflate3.hip (hipcc -S; the product flags).  A loop is classified by what it
writes: the speculative pass stores a checkpoint word (ds_write_b32), the emit three bytes
(ds_write_b8) and a bitmap bit (ds_or), the re-decode reads the next checkpoint (ds_read_b32) and
the warm-up none of these.  Only loops with two global loads (the two refills of a decode step)
and the common-path (non-SLOW) instantiation are listed.

  python tools/isa_loops.py [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.environ.get('DQ_ISA_SRC', os.path.join(ROOT, 'disq_amd', 'csrc', 'dq_inflate3.hip'))


def isa(flags):
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "-munsafe-fp-atomics", "-I" + os.path.join(ROOT, "include"), "-mllvm",
           "-amdgpu-sched-strategy=max-ilp", "--cuda-device-only", "-S", "-o", out, SRC] + flags
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def kernel(text, prefix):
    lines = text.split("\n")
    a = next(i for i, l in enumerate(lines) if l.startswith(prefix))
    b = next(i for i in range(a, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[a:b]


def loops(lines):
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):.*Depth=(\d+)", l)
        if not m:
            continue
        name = m.group(1)
        last = None
        for j in range(i + 1, min(len(lines), i + 900)):
            if re.search(r"s_(cbranch_\w+|branch)\s+" + re.escape(name) + r"$", lines[j].strip()):
                last = j
        if last is None:
            continue
        body = [x.strip() for x in lines[i + 1:last + 1]
                if x.strip() and not x.strip().startswith((";", "."))]
        yield name, body


def classify(body):
    has = lambda op: any(x.startswith(op) for x in body)  # noqa: E731
    if has("ds_write_b8") and has("ds_or"):
        return "emit"
    if has("ds_write_b32"):
        return "spec"
    if has("ds_read_b32"):
        return "redo"
    return "warm-up"


def main():
    text = isa(sys.argv[1:])
    ker = kernel(text, "_ZN2dq12_GLOBAL__N_120inflate_block_kernelILb0")
    seen = {}
    for name, body in loops(ker):
        g = sum(x.startswith("global_load") for x in body)
        if g != 2 or any(x.startswith("v_bfrev_b32") for x in body):
            continue  # not a decode step, or the canonical (SLOW) instantiation
        v = sum(x.startswith("v_") for x in body)
        s = sum(x.startswith("s_") for x in body)
        d = sum(x.startswith("ds_") for x in body)
        kind = classify(body)
        if kind not in seen or v < seen[kind][1]:
            seen[kind] = (name, v, s, d)
    for k in ("warm-up", "spec", "redo", "emit"):
        if k in seen:
            name, v, s, d = seen[k]
            print(f"{k:8s} {name:12s} VALU {v:4d}  SALU {s:4d}  DS {d:3d}")


if __name__ == "__main__":
    main()
