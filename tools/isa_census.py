"""ISA census of one kernel from a hipcc --save-temps .s file: per basic block, the count of
VALU / packed VALU / MFMA / LDS / global / scalar / wait instructions and the block's
branch target (a backward branch marks a loop).  Used to attribute VALU work per phase.

    python tools/isa_census.py FILE.s SYMBOL [--blocks]
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(("v_div_", "v_rcp", "v_sqrt", "v_rsq")):
        return "valu_trans_div"
    if op.startswith("v_cndmask"):
        return "valu_cndmask"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "valu_cmp"
    if op.startswith(("v_permlane", "v_mov_b32_dpp", "v_readlane", "v_readfirstlane", "v_writelane")):
        return "valu_xlane"
    if op.startswith(("v_lshl_add_u64", "v_lshlrev_b64", "v_add_co", "v_addc_co", "v_mad_u64", "v_ashrrev_i32", "v_mul_lo", "v_mul_hi", "v_lshl_add_u32", "v_add_u32", "v_lshlrev_b32", "v_and_b32", "v_or_b32", "v_mad_u32", "v_sub_u32", "v_bfe")):
        return "valu_int"
    if op.startswith("v_"):
        return "valu_fp"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def census(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = {"c": Counter(), "ops": Counter(), "line": start, "br": []}
    for i in range(start + 1, end):
        l = lines[i].split(";")[0].strip()
        if not l or l.startswith("."):
            m = re.match(r"^(\.LBB[\w_]+):", l)
            if m:
                cur = m.group(1)
                blocks[cur] = {"c": Counter(), "ops": Counter(), "line": i, "br": []}
            continue
        op = l.split()[0]
        blocks[cur]["c"][classify(op)] += 1
        blocks[cur]["ops"][op] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            blocks[cur]["br"].append(l.split()[-1])
    return blocks


if __name__ == "__main__":
    path, sym = sys.argv[1], sys.argv[2]
    b = census(path, sym)
    order = list(b)
    tot = Counter()
    for k, v in b.items():
        tot.update(v["c"])
        if "--blocks" in sys.argv:
            back = [t for t in v["br"] if t in b and order.index(t) <= order.index(k)]
            print(f"{k:28s} line {v['line']:7d} " + " ".join(f"{c}={n}" for c, n in sorted(v['c'].items()))
                  + (f"  LOOP->{back}" if back else ""))
    print("total", dict(tot))
