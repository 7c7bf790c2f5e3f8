"""Summarise a kernel's instruction stream from a hipcc -S file: python tools/asm_loop.py file.s NAME_SUBSTR
Prints run-length-compressed opcode sequence (waitcnt / barrier / ds / mfma / buffer / global / branch), with labels."""
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    if l.startswith("_Z") and sub in l and l.rstrip().endswith(":") is False and ":" in l and "@" in l:
        start = i
        break
    if l.startswith("_Z") and sub in l and l.split(";")[0].strip().endswith(":"):
        start = i
        break
if start is None:
    sys.exit("not found")
print(lines[start][:120])
out = []
for l in lines[start + 1:]:
    if l.startswith("\t.section") or l.startswith(".Lfunc_end"):
        break
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        if s.startswith(".LBB"):
            out.append(s.split(";")[0])
        continue
    op = s.split()[0]
    keep = ("s_waitcnt" in op or "barrier" in op or op.startswith("ds_") or "mfma" in op or op.startswith("buffer_")
            or op.startswith("global_") or op.startswith("s_cbranch") or op.startswith("s_branch") or "setprio" in op
            or op.startswith("s_sleep") or op.startswith("scratch_"))
    if keep:
        out.append(s if "waitcnt" in op else op)
# run-length compress
prev, n = None, 0
res = []
for o in out:
    if o == prev:
        n += 1
    else:
        if prev is not None:
            res.append(f"{prev} x{n}" if n > 1 else prev)
        prev, n = o, 1
res.append(f"{prev} x{n}" if n > 1 else prev)
print("\n".join(res))
