"""Kernel timings of the float-path matcher on bench.bench_matcher_float's workload, with no
parity guard: for tuning builds of the library (VO_LIB_PATH=...; timing-only variants are patches
applied outside the product sources).  Prints one JSON line: HIP-event microseconds per kernel."""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from visualodometry_amd import _lib, matcher  # noqa: E402
from visualodometry_amd.synthetic import superpoint_like_pair  # noqa: E402

batch, n, dim, calls = 16, 2048, 256, 10
ctx = _lib.context(0)
pairs = [superpoint_like_pair(n, n, 2000 + b, dim=dim) for b in range(batch)]
matcher.set_descriptor_kind(matcher.DESC_FLOAT, ctx)
a = _lib.DeviceArray.from_numpy(ctx, np.stack([q[0] for q in pairs]))
b = _lib.DeviceArray.from_numpy(ctx, np.stack([q[1] for q in pairs]))
out = _lib.DeviceArray(ctx, (batch, n), np.int32)
for _ in range(2):
    matcher.match_batch_device(a, b, out=out, ctx=ctx)
matcher.synchronize(ctx)
_lib.profile_enable(ctx, True)
for _ in range(calls):
    matcher.match_batch_device(a, b, out=out, ctx=ctx)
matcher.synchronize(ctx)
prof = _lib.profile_read(ctx)
_lib.profile_enable(ctx, False)
print(json.dumps({k: round(v[0] / v[1] * 1e3, 2) for k, v in prof.items()}))
