#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing (development aid):
counts by class for the function body.  Usage: isa_mix.py <file.s> <symbol>"""
import collections
import re
import sys

src, sym = sys.argv[1], sys.argv[2]
text = open(src).read()
i = text.index("\n" + sym + ":")
j = text.index(".Lfunc_end", i)
body = text[i:j].splitlines()
cnt = collections.Counter()
ops = collections.Counter()
for ln in body:
    ln = ln.strip()
    if not ln or ln.startswith((";", ".", "_")) or ln.endswith(":"):
        continue
    op = ln.split()[0]
    ops[op] += 1
    if op.startswith("v_fma_f64") or op.startswith("v_mul_f64") or op.startswith("v_add_f64"):
        cnt["fp64"] += 1
    elif op.startswith("v_readlane"):
        cnt["readlane"] += 1
    elif op.startswith("v_"):
        cnt["other_valu"] += 1
    elif op.startswith("ds_"):
        cnt["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cnt["vmem"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        cnt["branch"] += 1
    elif op.startswith("s_"):
        cnt["salu"] += 1
print(sym, sum(ops.values()), "instructions (static)")
for k, v in cnt.most_common():
    print(f"  {k:12s} {v}")
print("top opcodes:")
for k, v in ops.most_common(40):
    print(f"  {k:28s} {v}")
