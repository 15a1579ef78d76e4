"""Source check of a gfx950 store-data hazard the compiler misses: a MUBUF store of
more than 8 B (buffer_store_dwordx3/x4) reads its data VGPRs a cycle late, and ROCm 7.2's LLVM inserts the
wait state before a VALU write of those VGPRs only when the store's soffset is not a register.  On gfx950 the
write corrupts the stored data either way (measured: ~0.1 % of the SoC pair slots at 65,536 envs with an SGPR
soffset).  So every wide raw-buffer store in the kernels passes a literal 0 soffset and carries its uniform
offset in the V# base."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "smart-nanogrid-gym_amd", "csrc", "sng_kernels.hip")


def test_wide_buffer_stores_use_a_zero_soffset():
    text = open(SRC).read()
    calls = [m.start() for m in re.finditer(r"__builtin_amdgcn_raw_buffer_store_b(96|128)\s*\(", text)]
    assert calls, "no wide buffer stores found"
    for pos in calls:
        depth, i = 0, text.index("(", pos)
        args, cur = [], ""
        while True:
            ch = text[i]
            if ch == "(":
                depth += 1
                if depth > 1:
                    cur += ch
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    args.append(cur.strip())
                    break
                cur += ch
            elif ch == "," and depth == 1:
                args.append(cur.strip())
                cur = ""
            else:
                cur += ch
            i += 1
        line = text.count("\n", 0, pos) + 1
        assert len(args) == 5 and args[3] == "0", f"sng_kernels.hip:{line}: soffset {args[3]!r} (must be 0)"
