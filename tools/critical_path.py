"""Main-stream (critical-path) busy fraction of a C4 register_scan stream from a
rocprofv3 kernel trace (bench.py run under `rocprofv3 --kernel-trace`).

  python tools/critical_path.py <kernel_trace.csv> <timed_steps> [out.json] [skip]

register_scan's critical path is the context stream: match -> pair scatter -> window
linearization -> host LM turn-around -> ...  The pipelined extraction (side2) and the
speculative map build (side) run beside it.  Over the last `timed_steps` scans of the
trace (one k_extract_rows per scan), this reports the union of the context stream's
kernel intervals over the wall span: the fraction of the scan the critical path keeps
the GPU busy; the rest is host time (LM solves, launch and completion-word latency).
skip: scans at the end of the trace to leave out (bench.py's profile pass follows its
timed steps: skip = --steps selects the timed ones).
Streams come from the trace's Stream_Id column when present, else from kernel names
(extraction and map-build kernels are the side streams' in the pipelined bench).
"""
import csv
import os
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import provenance  # noqa: E402

SIDE = re.compile(r"k_extract_rows|k_normals|k_row_blocks|k_closest|k_fit|k_write_features|k_row_scan|k_scan_|k_map_")


def short(n):
    m = re.search(r"(k_\w+|__amd_rocclr_\w+)", n)
    return m.group(1) if m else n[:40]


def main():
    path, timed = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    sid_col = next((c for c in ("Stream_Id", "Queue_Id") if rows and c in rows[0]), None)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 r.get(sid_col) if sid_col else None) for r in rows)
    starts = [i for i, e in enumerate(ev) if e[2] == "k_extract_rows"]
    if len(starts) < timed + 1:
        raise SystemExit(f"trace holds {len(starts)} scans, fewer than {timed} + 1")
    # the context stream: the stream of the k_match launches
    main_sid = None
    if sid_col:
        cnt = defaultdict(int)
        for e in ev:
            if e[2] == "k_match":
                cnt[e[3]] += 1
        main_sid = max(cnt, key=cnt.get) if cnt else None

    def is_main(e):
        return e[3] == main_sid if main_sid is not None else not SIDE.search(e[2])

    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    if len(starts) < timed + skip + 1:
        raise SystemExit(f"trace holds {len(starts)} scans, fewer than {timed} + {skip} + 1")
    a, b = starts[-timed - skip - 1], starts[-skip - 1]
    t0, t1 = ev[a][0], ev[b][0]
    busy, last = 0, t0
    per = defaultdict(float)
    for s, e, n, sid in ev:
        if s < t0 or s >= t1 or not is_main((s, e, n, sid)):
            continue
        e2 = min(e, t1)
        if e2 > last:
            busy += e2 - max(s, last)
            last = e2
        per[n] += (e - s) / 1e3 / timed
    span = (t1 - t0) / 1e3
    out = {"timed_scans": timed, "span_us_per_scan": round(span / timed, 2),
           "main_stream_busy_us_per_scan": round(busy / 1e3 / timed, 2),
           "main_stream_busy_frac": round(busy / 1e3 / span, 4),
           "stream_source": sid_col or "kernel names",
           "main_stream_kernels_us_per_scan": {k: round(v, 2) for k, v in sorted(per.items(), key=lambda x: -x[1])}}
    print(json.dumps(out, indent=1))
    out["skipped_trailing_scans"] = skip
    provenance.stamp(out)  # the sources this run measured (bench.py marks stale profiles)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
