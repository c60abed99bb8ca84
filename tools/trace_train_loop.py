"""Which kernels run between the training steps of train_byol.py's loop: reads a
rocprofv3 --kernel-trace CSV of the CLI (tools/trace_train_loop.sh) and, inside the window from
the first to the last AdamW dispatch of the epoch (the training steps; validation and checkpointing
come after it), counts the dispatches that are not this library's kernels -- ATen
(at::native / FillFunctor / elementwise), runtime blits (__amd_rocclr_copyBuffer / fillBuffer).
Usage: python tools/trace_train_loop.py gpurun_out/DIR/run_kernel_trace.csv [steps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start_Time"
key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End_Time"
rows.sort(key=lambda r: int(r[key_s]))
adam = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
lo, hi = adam[0], adam[-1]
foreign = collections.Counter()
ours = collections.Counter()
for r in rows[lo:hi + 1]:
    n = r["Kernel_Name"]
    if "at::" in n or "rocclr" in n or "FillFunctor" in n or "elementwise" in n or "Reduce" in n:
        foreign[n[:110]] += 1
    else:
        ours[n.split("(")[0][-60:]] += 1
span_ms = (int(rows[hi][key_e]) - int(rows[lo][key_s])) / 1e6
print(f"training window: {hi - lo + 1} dispatches, {span_ms:.1f} ms, {len(adam)} AdamW dispatches"
      + (f", {steps} steps" if steps else ""))
print(f"non-library dispatches in the window: {sum(foreign.values())}")
for n, c in foreign.most_common():
    print(f"  {c:5d}  {n}")
outside = collections.Counter(r["Kernel_Name"][:110] for r in rows[:lo] + rows[hi + 1:]
                              if "at::" in r["Kernel_Name"] or "rocclr" in r["Kernel_Name"])
print(f"(outside the window -- model build, first batch, validation, checkpoint: {sum(outside.values())})")
