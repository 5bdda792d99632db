"""Scan gfx950 device assembly for cross-lane reads too close to the VALU write of their
operand (DPP src0 / v_permlane*_swap operands need 2 wait states after it).

The compiler inserts these wait states for the cross-lane instructions it emits itself but
cannot see inside inline asm; hdgnn.hip's row16_sums / swap helpers carry their own
s_nop.  A violation reads the operand's previous value on some lanes: silently wrong sums
that depend on the schedule (how the round-2 pair_tile32 "wrong pass B" results arose).

    python tools/dpp_hazards.py file.s [...]          # prints violations, exit 1 if any
"""
import re
import sys

_VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def _regs(tok):
    m = _VREG.fullmatch(tok.strip())
    if not m:
        return []
    if m.group(3) is not None:
        return [int(m.group(3))]
    return list(range(int(m.group(1)), int(m.group(2)) + 1))


def _operands(text):
    parts = text.split(None, 1)
    return [] if len(parts) < 2 else [o.strip() for o in parts[1].split(",")]


def _reads(op, text):
    """VGPRs the cross-lane instruction reads from other lanes, or None."""
    ops = _operands(text)
    if op.startswith("v_permlane") and op.endswith("_swap_b32"):
        return set(_regs(ops[0]) + _regs(ops[1]))
    if op.endswith("_dpp") and len(ops) >= 2:
        return set(_regs(ops[1]))
    return None


def _writes(op, text):
    if not op.startswith("v_") or op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    ops = _operands(text)
    return set(_regs(ops[0])) if ops else set()


def scan(path):
    fn, stream, bad = None, [], []
    for line in open(path):
        s = line.split(";")[0].strip()
        if not s or s.startswith((".", "//")) and not s.endswith(":"):
            continue
        if s.endswith(":"):
            if not s.startswith(".L"):
                fn = s[:-1]
            stream.append(None)                 # control may join here: stop looking back
            continue
        stream.append((fn, s))
    for k, ins in enumerate(stream):
        if ins is None:
            continue
        op = ins[1].split()[0]
        rd = _reads(op, ins[1])
        if not rd:
            continue
        ws, j = 0, k - 1
        while j >= 0 and ws < 2 and stream[j] is not None:
            prev = stream[j][1]
            pop = prev.split()[0]
            if pop == "s_nop":
                ws += int(prev.split()[1], 0) + 1
            else:
                if _writes(pop, prev) & rd:
                    bad.append((ins[0], prev, ins[1], ws))
                    break
                ws += 1
            j -= 1
    return bad


def main(paths):
    n = 0
    for p in paths:
        for fn, w, r, ws in scan(p):
            n += 1
            print("%s: %s\n    %s  -> %s  (%d wait states)" % (p, fn, w, r, ws))
    return 1 if n else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
