"""bench.py's roofline bookkeeping, without a GPU: every committed PMC profile the bench
would pick for a workload holds counters for that workload's kernels (the families the
launchers time, including the persistent renders and their folds), and the family
patterns do not mix kernels of different families."""
import glob
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    pytest.importorskip("torch")
    sys.path.insert(0, ROOT)
    import bench as b  # noqa: E402  (imports torch and rtmi; no GPU call)

    return b


def test_family_patterns_separate_the_kernels(bench):
    keys = ["k_render_ps<0, 0, 1>", "k_render<1, 0, 1, true, false, 4>", "k_render_pq<0, 1, 4>", "k_fold_chunks",
            "k_sarsa_render<1, 0>", "k_sarsa_render_pq<1, 0>", "k_sarsa_fold", "k_sarsa_apply",
            "k_dqn_mlp<4, false>", "k_dqn_bounce<4, false>", "k_dqn_camera<4>"]

    def pick(kernel):
        return sorted(k for k in keys if re.search(bench.family_re(kernel), k))

    assert pick("k_render_ps<") == ["k_render_ps<0, 0, 1>"]
    assert pick("k_render<") == ["k_fold_chunks", "k_render<1, 0, 1, true, false, 4>", "k_render_pq<0, 1, 4>"]
    assert pick("k_sarsa_render<") == ["k_sarsa_fold", "k_sarsa_render<1, 0>", "k_sarsa_render_pq<1, 0>"]
    assert pick("k_sarsa_apply<") == ["k_sarsa_apply"]
    assert pick("k_dqn_mlp<") == ["k_dqn_mlp<4, false>"]
    assert pick("k_dqn_bounce<") == ["k_dqn_bounce<4, false>"]


def test_profile_table_matches_bench_frames(bench):
    """tools/bench_pmc_summary.py keys profiles by the frame it ran: its frame defaults are
    bench.py's, and every profiled command parses to the frame bench.py would match"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_pmc_summary as bps
    for wl, (_, _, _, W, H, spp, split, _) in bench.WORKLOADS.items():
        assert bps.BENCH_FRAMES[wl] == (W, H, spp, split)
    for name, (_, _, _, args, scale) in bps.WORKLOADS.items():
        wl, *frame = bps.frame_of_args(args)
        prof = {"workload_name": wl, "command": "python3 bench.py " + args}
        assert bench.profile_frame(prof) == tuple(frame), name
        assert scale in (1, 2)
    assert bps.WORKLOADS["door_room_sarsa"][4] == 1  # gathers: FETCH_SIZE not doubled


@pytest.mark.parametrize("workload", ["cornell", "complex_light", "door_room_sarsa", "archway_dqn"])
def test_newest_profile_has_the_dominant_kernel(bench, workload):
    """the newest committed profile of each workload yields per-frame counters for the
    kernel its roofline divides by (a name change of a kernel would leave frac null)"""
    profs = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "*_bench_pmc.json")):
        p = json.load(open(path))
        if p.get("workload_name", "cornell") == workload and p.get("created"):
            profs.append((p["created"], path, p))
    assert profs, f"no committed profile for {workload}"
    _, path, prof = max(profs)
    kname = bench.ROOF[workload][1]
    per, _ = bench.frame_counters(prof, kname, prof.get("warmup", 0), prof.get("steps", 1))
    assert per.get("SQ_INSTS_VALU", 0) > 0, (path, kname)
    assert per.get("duration_ns", 0) > 0, (path, kname)
