"""Compress a kernel's gfx950 ISA into runs of the instructions that shape a K-loop schedule.

usage: python scripts/isa_summary.py FILE.s KERNEL_SUBSTRING [--all]

Prints one line per run of identical opcodes among s_waitcnt / s_barrier / ds_read / ds_write /
global_load_lds / buffer_load / v_mfma / branches / labels / s_setprio (``--all`` keeps every opcode), with
the line number of the run's first instruction and the operands of its last one.
"""
import re
import sys

KEEP = re.compile(r"^(s_waitcnt|s_barrier|ds_read|ds_write|global_load|buffer_load|buffer_store|global_store|v_mfma|"
                  r"s_cbranch|s_branch|s_setprio|s_endpgm|s_sleep)")


def main():
    path, name = sys.argv[1], sys.argv[2]
    keep_all = "--all" in sys.argv
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        head = ln.split(";")[0].rstrip()
        if head.endswith(":") and not head.startswith(".") and name in head:
            start = i
            break
    if start is None:
        sys.exit(f"kernel {name!r} not found")
    runs = []
    for i in range(start + 1, len(lines)):
        ln = lines[i].strip()
        if ln.startswith(".Lfunc_end"):
            break
        if ln.startswith(".LBB"):
            runs.append([ln, 1, "", i + 1])
            continue
        if not ln or ln.startswith((";", ".")):
            continue
        op = ln.split()[0]
        if not keep_all and not KEEP.match(op):
            continue
        args = ln[len(op):].split(";")[0].strip()
        if runs and runs[-1][0] == op:
            runs[-1][1] += 1
            runs[-1][2] = args
        else:
            runs.append([op, 1, args, i + 1])
    for op, n, args, ln in runs:
        print(f"{ln:6d} {op:40s} x{n:<3d} {args}")


if __name__ == "__main__":
    main()
