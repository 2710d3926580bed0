"""Repeat the DP-pipeline-vs-eager record comparison with slot-parallel on / off to tell
a race from a deterministic difference (usage: python scripts/debug_slot.py N)."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import test_hip_kernels as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for mode in ("0", "1"):
    os.environ["SSA_SLOT_PARALLEL"] = mode
    ok = 0
    for i in range(n):
        try:
            T.test_dp_pipeline_records_match_eager(1)
            ok += 1
        except AssertionError as e:
            print(f"slot={mode} run {i}: MISMATCH {str(e)[:200]}", flush=True)
    print(f"slot={mode}: {ok}/{n} match", flush=True)
