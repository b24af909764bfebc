"""Per-basic-block instruction counts of one kernel in a `hipcc -S` listing.

usage: python tools/asm_blocks.py file.s kernel_substring [min_insts]
Prints each block (label, VALU / SALU / LDS / VMEM / branch counts) and marks the
backward branches (loops) -- a quick map of where a kernel's issue slots go.
"""
import re
import sys


def main():
    path, ksub = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines)
              if re.match(r"^_Z\S*:", l) and ksub in l)
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, order = {}, "entry", ["entry"]
    blocks[cur] = []
    for l in lines[st + 1:en]:
        t = l.split(";")[0].strip()
        if not t or t.startswith("."):
            if re.match(r"^\.LBB\S*:", t):
                cur = t[:-1]
                blocks[cur] = []
                order.append(cur)
            continue
        blocks[cur].append(t)
    pos = {b: i for i, b in enumerate(order)}
    tot = {}
    for b in order:
        ins = blocks[b]
        c = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "smem": 0, "other": 0}
        back = []
        for t in ins:
            op = t.split()[0]
            if op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
            elif op.startswith("s_load") or op.startswith("s_buffer"):
                c["smem"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
                if op.startswith("s_cbranch") or op == "s_branch":
                    tgt = t.split()[-1]
                    if tgt in pos and pos[tgt] <= pos[b]:
                        back.append(tgt)
            else:
                c["other"] += 1
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        if len(ins) >= mn:
            print(f"{b:14s} n={len(ins):5d} valu={c['valu']:5d} salu={c['salu']:4d} "
                  f"lds={c['lds']:4d} vmem={c['vmem']:3d}" + (f"  LOOP->{back}" if back else ""))
    print("total", tot)


if __name__ == "__main__":
    main()
