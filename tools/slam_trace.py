#!/usr/bin/env python3
"""Reads slam_rate's event trace (YOUTH_SLAM_TRACE=<file>, youth_slam_trace_*)
and, optionally, the rocprofv3 kernel trace of the same run, and prints per
backlogged pass: the rate, the micro-batches the worker formed (sizes), where
the worker's time went (collect waits, submits, idle waits, the rest), the
producer's push time, and the longest GPU-idle gap with the worker and
producer events around it (which wait it sits in).

usage: slam_trace.py TRACE [KERNEL_TRACE_CSV]
       slam_trace.py --live TRACE.live [KERNEL_TRACE_CSV]
(--live: slam_rate's one-frame-at-a-time phase, "# live k t0 t1" windows:
the median time of each step of a frame from processSlamFrame's call to its
pose in the trajectory, and the tracker kernels' span inside it)
"""
import csv
import sys

KINDS = {1: "push_begin", 2: "push_end", 3: "take", 4: "submit_begin", 5: "submit_end",
         6: "collect_begin", 7: "collect_end", 8: "idle_begin", 9: "idle_end", 10: "pool",
         11: "drop", 12: "submit_step"}


def load(path):
    passes, ev = [], []
    with open(path) as f:
        for ln in f:
            if ln.startswith("# pass"):
                _, _, p, t0, t1 = ln.split()
                passes.append((float(t0), float(t1)))
            elif ln.strip():
                t, k, a = ln.split()
                ev.append((float(t), int(k), int(a)))
    return passes, ev


def kernels(path):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            out.append((int(row["Start_Timestamp"]) * 1e-9, int(row["End_Timestamp"]) * 1e-9,
                        row["Kernel_Name"][:40]))
    return sorted(out)


def spans(ev, begin, end):
    """(t_begin, t_end, arg_begin) of matched begin/end events."""
    out, open_t = [], None
    for t, k, a in ev:
        if k == begin:
            open_t = (t, a)
        elif k == end and open_t is not None:
            out.append((open_t[0], t, open_t[1]))
            open_t = None
    return out


def live(path, kt=None):
    wins, ev = [], []
    with open(path) as f:
        for ln in f:
            if ln.startswith("# live"):
                _, _, k, t0, t1 = ln.split()
                wins.append((float(t0), float(t1)))
            elif ln.strip():
                t, k, a = ln.split()
                ev.append((float(t), int(k), int(a)))
    ks = kernels(kt) if kt else None
    steps = {}

    def add(name, v):
        steps.setdefault(name, []).append(v * 1e6)
    for t0, t1 in wins[1:]:              # the first frame starts the sequence
        e = [x for x in ev if t0 <= x[0] <= t1]
        first = {}
        for t, k, a in e:
            first.setdefault(k, t)
        last = {}
        for t, k, a in e:
            last[k] = t
        if not all(k in first for k in (2, 4, 5, 6, 7)):
            continue
        add("total", t1 - t0)
        add("push (processSlamFrame copy)", first[2] - t0)
        add("push end -> worker submit", first[4] - first[2])
        add("submit (pull + launch enqueue)", first[5] - first[4])
        add("submit end -> collect begin", first[6] - first[5])
        add("collect (wait for the pose)", last[7] - first[6])
        add("collect end -> pose seen", t1 - last[7])
        if ks:
            kk = [x for x in ks if first[4] - 1e-4 <= x[0] <= t1]
            if kk:
                add("first kernel start - submit begin", kk[0][0] - first[4])
                add("kernels first start -> last end", max(x[1] for x in kk) - kk[0][0])
                add("last kernel end -> collect end", last[7] - max(x[1] for x in kk))
                for x in kk:
                    add("kernel " + x[2].split("(")[0].replace("void ", ""), x[1] - x[0])
    print(f"live frames: {len(wins) - 1} (median us per step)")
    for k, v in steps.items():
        v = sorted(v)
        print(f"  {k:42s} {v[len(v) // 2]:8.1f}   (p10 {v[len(v) // 10]:7.1f}, p90 {v[(9 * len(v)) // 10]:7.1f})")


def main():
    if sys.argv[1] == "--live":
        live(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
        return
    passes, ev = load(sys.argv[1])
    ks = kernels(sys.argv[2]) if len(sys.argv) > 2 else None
    for p, (t0, t1) in enumerate(passes):
        e = [x for x in ev if t0 <= x[0] <= t1]
        dur = t1 - t0
        takes = [a for _, k, a in e if k == 3]
        coll = spans(e, 6, 7)
        subm = spans(e, 4, 5)
        idle = spans(e, 8, 9)
        push = spans(e, 1, 2)
        pushes = [a for _, k, a in e if k == 2]
        worker = sorted([(b, c, "collect") for b, c, _ in coll] + [(b, c, "submit") for b, c, _ in subm] +
                        [(b, c, "idle") for b, c, _ in idle])
        line = (f"pass {p}: {300 if not push else len(push)} frames {len(push) / dur:8.0f} frames/s "
                f"{dur * 1e3:6.2f} ms | launches {len(subm)} sizes {sorted(takes)[:3]}..{sorted(takes)[-3:]} | "
                f"worker collect {sum(c - b for b, c, _ in coll) * 1e3:5.2f} ms (max {max([c - b for b, c, _ in coll] or [0]) * 1e3:.2f}) "
                f"submit {sum(c - b for b, c, _ in subm) * 1e3:5.2f} ms (max {max([c - b for b, c, _ in subm] or [0]) * 1e3:.2f}) "
                f"idle {sum(c - b for b, c, _ in idle) * 1e3:5.2f} ms | producer push {sum(c - b for b, c, _ in push) * 1e3:5.2f} ms "
                f"(max {max([c - b for b, c, _ in push] or [0]) * 1e3:.2f}), new buffers {sum(1 for a in pushes if a)}")
        print(line)
        # the longest stretch of the worker not inside a traced call, and the
        # longest single traced call
        gaps = [(worker[i + 1][0] - worker[i][1], worker[i][1], worker[i][2], worker[i + 1][2])
                for i in range(len(worker) - 1)]
        if gaps:
            g = max(gaps)
            print(f"    worker: longest untraced stretch {g[0] * 1e3:.3f} ms at +{(g[1] - t0) * 1e3:.2f} ms "
                  f"(after {g[2]}, before {g[3]})")
        if worker:
            w = max(worker, key=lambda x: x[1] - x[0])
            print(f"    worker: longest call {w[2]} {(w[1] - w[0]) * 1e3:.3f} ms at +{(w[0] - t0) * 1e3:.2f} ms")
        # submissions over 1 ms: the time to each step inside them
        cur = None
        for t, k, a in e:
            if k == 4:
                cur = [t, a, []]
            elif k == 12 and cur:
                cur[2].append((a, t))
            elif k == 5 and cur:
                if t - cur[0] > 1e-3:
                    steps = ", ".join(f"step {a} +{(ts - cur[0]) * 1e3:.3f}" for a, ts in cur[2])
                    print(f"    slow submit of {cur[1]} frames at +{(cur[0] - t0) * 1e3:.2f} ms: "
                          f"{(t - cur[0]) * 1e3:.3f} ms ({steps})")
                cur = None
        if ks:
            kk = [x for x in ks if x[1] >= t0 and x[0] <= t1]
            if len(kk) > 1:
                gi = max(range(len(kk) - 1), key=lambda i: kk[i + 1][0] - kk[i][1])
                g0, g1 = kk[gi][1], kk[gi + 1][0]
                print(f"    GPU: {len(kk)} kernels, longest idle gap {(g1 - g0) * 1e3:.3f} ms at "
                      f"+{(g0 - t0) * 1e3:.2f} ms; events inside it:")
                for t, k, a in e:
                    if g0 - 2e-4 <= t <= g1 + 2e-4:
                        print(f"      +{(t - t0) * 1e3:8.3f} ms {KINDS.get(k, k):14s} {a}")


if __name__ == "__main__":
    main()
