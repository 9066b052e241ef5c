"""Attribute device copies (hipMemcpy*/copyBuffer) in a torch.profiler chrome trace to the innermost
enclosing CPU op on the same thread.  Usage: python tools/trace_copies.py trace.json"""
import collections
import json
import sys

ev = [e for e in json.load(open(sys.argv[1]))["traceEvents"] if e.get("ph") == "X"]
ops = [e for e in ev if e.get("cat") in ("cpu_op", "user_annotation", "python_function")]
rt = [e for e in ev if e.get("cat") in ("cuda_runtime", "hip_runtime") and "emcpy" in e.get("name", "")]
by_tid = collections.defaultdict(list)
for o in ops:
    by_tid[o["tid"]].append(o)
cnt = collections.Counter()
for r in rt:
    best = None
    for o in by_tid.get(r["tid"], ()):
        if o["ts"] <= r["ts"] and r["ts"] + r.get("dur", 0) <= o["ts"] + o.get("dur", 0):
            if best is None or o.get("dur", 0) < best.get("dur", 0):
                best = o
    cnt[(r["name"], best["name"] if best else "?")] += 1
kern = collections.Counter(e["name"][:60] for e in ev if e.get("cat") == "kernel" and "opy" in e["name"])
print("runtime copy calls by enclosing op:")
for (n, o), c in cnt.most_common(25):
    print(f"  {c:5d}  {n:28s} <- {o}")
print("copy kernels:", dict(kern))
