#!/usr/bin/env python3
"""Static check of hand-counted VMEM loads in a kernel's ISA (hipcc -S).

Walks one function in layout order, keeping the destination registers of
outstanding global/buffer loads in issue order; `s_waitcnt vmcnt(N)` retires
all but the newest N.  Any other instruction that reads or writes a register
of an outstanding load is reported (a copy the compiler placed between an
inline-asm load and the wait that lands it would read stale data).  Layout
order approximates control flow; a report is a lead to read the ISA, not a
proof.  usage: check_asm_loads.py file.s function_name
"""
import re
import sys


def regs(text):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path, fn):
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    pending = []  # [(line, set(dest regs))] oldest first
    bad = 0
    for i in range(st, en):
        s = lines[i].split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", s)
        if m:
            n = int(m.group(1))
            if len(pending) > n:
                pending = pending[len(pending) - n:] if n else []
            continue
        if op.startswith("s_endpgm"):
            pending = []
            continue
        args = s[len(op):]
        busy = set().union(*[p[1] for p in pending]) if pending else set()
        touched = regs(args)
        if op.startswith(("global_load", "buffer_load")) and " lds" not in s:
            dst = regs(args.split(",")[0])
            hit = (touched - dst) & busy | (dst & busy)
            if hit:
                print(f"{i + 1}: {s}   <- outstanding {sorted(hit)[:8]}")
                bad += 1
            pending.append((i, dst))
            continue
        if touched & busy:
            print(f"{i + 1}: {s}   <- outstanding {sorted(touched & busy)[:8]}")
            bad += 1
    print(f"{fn}: {bad} accesses to registers of outstanding loads")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
