"""Per-kernel summary of the last single-image SIFT call in a rocprofv3 kernel trace database
(``rocprofv3 --kernel-trace -- python3 tools/sift_single.py``): usage
``python tools/sift_trace_summary.py <results.db>`` -> JSON of kernel -> [launches, us]."""
import collections
import json
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
first = [i for i, r in enumerate(rows) if "sift_upsample_kernel" in r[0]][-1]
last = rows[first:]
agg = collections.OrderedDict()
for name, s, e in last:
    m = re.search(r"(sift_\w+|merge_sort\w*|radix_sort\w*|fillBuffer\w*|copyBuffer\w*)", name)
    k = m.group(1) if m else "rocprim other"
    a = agg.setdefault(k, [0, 0.0])
    a[0] += 1
    a[1] = round(a[1] + (e - s) / 1e3, 2)
out = {"kernels": agg, "span_us": round((last[-1][2] - last[0][1]) / 1e3, 1),
       "busy_us": round(sum(e - s for _, s, e in last) / 1e3, 1)}
print(json.dumps(out, indent=1))
