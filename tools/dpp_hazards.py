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


_BRANCH = re.compile(r"^s_(branch|cbranch_\w+)\s+(\S+)")


def _blocks(path):
    """Basic blocks of the assembly: (function, label, [instructions], successor labels).
    A block ends at a label or after a branch / s_endpgm; a conditional branch has the
    branch target and the fall-through as successors."""
    blocks, cur = [], None
    fn, anon = None, 0

    def open_block(label):
        nonlocal cur
        cur = {"fn": fn, "label": label, "ins": [], "succ": None}
        blocks.append(cur)

    for line in open(path):
        s = line.split(";")[0].strip()
        if not s or s.startswith((".", "//")) and not s.endswith(":"):
            continue
        if s.endswith(":"):
            if not s.startswith(".L"):
                fn = s[:-1]
                open_block(None)                  # a function entry: no predecessors
                cur["entry"] = True
            else:
                prev = cur
                open_block(s[:-1])
                if prev is not None and prev["succ"] is None:
                    prev["succ"] = [s[:-1]]       # falls through into the label
            continue
        if cur is None:
            open_block(None)
        cur["ins"].append((fn, s))
        op = s.split()[0]
        m = _BRANCH.match(s)
        if m or op in ("s_endpgm", "s_setpc_b64"):
            if op == "s_branch":
                cur["succ"] = [m.group(2)]
            elif m:                               # conditional: target + fall-through
                anon += 1
                nxt = ".Lfall%d" % anon
                cur["succ"] = [m.group(2), nxt]
                open_block(nxt)
                continue
            else:
                cur["succ"] = []
            open_block(".Lafter%d" % anon)
            anon += 1
    for b in blocks:
        if b["succ"] is None:
            b["succ"] = []
    return blocks


def scan(path):
    """Cross-lane reads (DPP src0, permlane swaps) with < 2 wait states after a VALU write
    of an operand, looking back across block boundaries into every predecessor
    (fall-through and branches, loop back-edges included)."""
    blocks = _blocks(path)
    by_label = {b["label"]: b for b in blocks if b["label"]}
    preds = {id(b): [] for b in blocks}
    for b in blocks:
        for t in b["succ"]:
            if t in by_label:
                preds[id(by_label[t])].append(b)
    bad = []

    def walk(b, j, ws, rd, ins, seen):
        """Look back from instruction j of block b with ws wait states already counted."""
        while j >= 0 and ws < 2:
            prev = b["ins"][j][1]
            pop = prev.split()[0]
            if pop == "s_nop":
                ws += int(prev.split()[1], 0) + 1
            elif _BRANCH.match(prev):
                pass                              # counted as no wait state (conservative)
            else:
                if _writes(pop, prev) & rd:
                    bad.append((ins[0], prev, ins[1], ws))
                    return
                ws += 1
            j -= 1
        if ws >= 2:
            return
        for p in preds[id(b)]:
            key = (id(p), ws)
            if key not in seen:
                seen.add(key)
                walk(p, len(p["ins"]) - 1, ws, rd, ins, seen)

    for b in blocks:
        for k, ins in enumerate(b["ins"]):
            op = ins[1].split()[0]
            rd = _reads(op, ins[1])
            if rd:
                walk(b, k - 1, 0, rd, ins, set())
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
