"""bench.py's rank launch: --gpus N without a launcher starts N ranks under
torch.distributed.run; under a launcher --gpus must equal WORLD_SIZE; the JSON line's n_gpus is the
live group's size.  Rehearsed on CPU with gloo (--launch-check: rank plumbing + frame-end gather)."""
import json
from pathlib import Path
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_launch_plan():
    assert bench.launch_plan(0, {}) == ("rank", 1)
    assert bench.launch_plan(1, {}) == ("rank", 1)
    assert bench.launch_plan(4, {}) == ("spawn", 4)
    assert bench.launch_plan(0, {"WORLD_SIZE": "8"}) == ("rank", 8)
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == ("rank", 8)
    with pytest.raises(SystemExit):
        bench.launch_plan(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.launch_plan(8, {"WORLD_SIZE": "2"})


def _run(args, timeout=240):
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


def test_gpus_2_spawns_two_gloo_ranks():
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_gathered"] == [0, 1]


def test_gpus_beyond_visible_devices_fails_loudly():
    # this container has no GPU: asking for 2 ranks of real work must fail before any rank starts
    if bench.visible_gpu_count() >= 2:
        pytest.skip("two or more devices visible")
    r = _run(["--gpus", "2", "--steps", "1"], timeout=120)
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr


def test_roofline_traffic_only_from_a_profile_of_the_same_config(tmp_path):
    """roofline.traffic / l2 / latency come from the newest committed PMC profile whose workload is
    the line's config field for field: a 1-spp, unordered or whole-frame profile
    never stands in for the timed 1040-spp ordered launch or a rank's share."""
    cfg = {"workload": "C3", "triangles": 10_000_002, "width": 1920, "height": 1080, "spp_per_step": 52,
           "spp": 1040, "form": "k_path", "ordered_fetch": True, "parallelism": "tile-split x1"}
    rec = {"hbm_bytes_per_spp": 11.5e9, "l2_req_bytes_per_spp": 40e9, "counters": {"VmemLatency": 900.0},
           "grid_threads": 262144}
    for tag, w in (("r01", cfg), ("r02", dict(cfg, ordered_fetch=False)), ("r03", dict(cfg, spp=20)),
                   ("r04", dict(cfg, extra=1))):
        (tmp_path / f"{tag}_traffic.json").write_text(json.dumps({"workload": w, "kernels": {"k_path<false, true>": rec}}))
    prof, src = bench.measured_traffic(bench.PATH_KERNEL_PROF_NAME, cfg, spp=1040, profiles_dir=tmp_path)
    assert src == "profiles/r01_traffic.json"
    assert prof["traffic"] == 11.5e9 * 1040 and prof["l2_bytes"] == 40e9 * 1040
    # a rank share, an unordered launch or another spp matches nothing
    for other in (dict(cfg, parallelism="tile-split x8"), dict(cfg, ordered_fetch=False, spp=7), dict(cfg, triangles=5)):
        assert bench.measured_traffic(bench.PATH_KERNEL_PROF_NAME, other, spp=1040, profiles_dir=tmp_path) == (None, None)
    # the latency model of the line
    cl = {"rays": 4, "visits": 100, "leaf_tests": 20}
    sh = {"rays": 1, "visits": 20, "leaf_tests": 5}
    lat = bench.latency_model(prof, cl, sh, 1, 1e9)
    assert lat["dependent_rounds_per_sample"] == 150
    assert abs(lat["ceiling_samples_per_s"] - 262144 / (150 * 900 / bench.SCLK_HZ)) < 1
    assert 0 < lat["frac"] < 1


def test_visible_gpu_count_from_sysfs(tmp_path):
    """Devices are counted from the KFD topology (gpu_id != 0: CPU nodes have 0), narrowed by the
    visibility variables, without torch or HIP."""
    for i, gid in enumerate((0, 4242, 0, 777, 999)):
        (tmp_path / str(i)).mkdir()
        (tmp_path / str(i) / "gpu_id").write_text(f"{gid}\n")
    (tmp_path / "9").mkdir()   # a node without gpu_id is skipped
    assert bench.visible_gpu_count({}, tmp_path) == 3
    assert bench.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,1"}, tmp_path) == 2
    assert bench.visible_gpu_count({"ROCR_VISIBLE_DEVICES": ""}, tmp_path) == 0
    assert bench.visible_gpu_count({}, tmp_path / "missing") == 0


def test_spawn_path_never_initialises_the_gpu_in_the_parent():
    """--gpus N's launcher counts devices and starts the ranks without importing torch.cuda state or
    loading the HIP runtime into the parent (exec after GPU init takes the machine down on the pool):
    the parent's memory map holds no libamdhip64 and torch is never imported."""
    code = f"""
import sys
sys.path.insert(0, {str(ROOT)!r})
import bench
bench.visible_gpu_count = lambda *a, **k: 2   # the count itself is tested separately
rc = bench.spawn_ranks(2, ["--launch-check"], need_devices=True)
maps = open("/proc/self/maps").read()
assert rc == 0, rc
assert "libamdhip64" not in maps, "HIP runtime loaded in the launcher"
assert "torch" not in sys.modules, "torch imported in the launcher"
print("LAUNCHER-CLEAN")
"""
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env,
                       cwd=str(ROOT))
    assert r.returncode == 0 and "LAUNCHER-CLEAN" in r.stdout, r.stderr[-3000:]


def _share_worker(rank, world, port, shm_dir, out_dir, fallback=None):
    import os as _os
    import torch.distributed as dist
    import numpy as _np
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(ROOT))
    import bench as b
    from akari_amd import capi
    nodes = _np.zeros(5, capi.NODE_DTYPE)
    nodes["axis"] = _np.arange(5)
    tris = _np.zeros(3, capi.TRI_DTYPE)
    tris["gid"] = [7, 8, 9]
    calls = []
    info = b.build_once_per_node(rank, build=lambda: calls.append("build") or "built", export=lambda: (nodes, tris),
                                 adopt=lambda n, t: calls.append("adopt") or (n.tobytes() == nodes.tobytes() and
                                                                              t.tobytes() == tris.tobytes()),
                                 barrier=dist.barrier, tag="t", shm_dir=Path(shm_dir),
                                 fallback_dirs=None if fallback is None else [Path(d) for d in fallback])
    dist.barrier()
    Path(out_dir, f"r{rank}").write_text(f"{info}|{','.join(calls)}")
    dist.destroy_process_group()


def test_bvh_built_once_per_node(tmp_path):
    """bench.py's multi-rank setup: rank 0 builds and shares the BVH2 through shared-memory files,
    the other ranks adopt an identical copy, and the files are removed afterwards (gloo, 3 ranks)."""
    import torch.multiprocessing as mp
    shm, out = tmp_path / "shm", tmp_path / "out"
    shm.mkdir()
    out.mkdir()
    mp.spawn(_share_worker, args=(3, bench._free_port(), str(shm), str(out)), nprocs=3, join=True)
    assert (out / "r0").read_text() == "built|build"
    assert (out / "r1").read_text() == (out / "r2").read_text() == "True|adopt"
    assert list(shm.iterdir()) == []


def test_bvh_share_falls_back_when_shm_has_no_room(tmp_path):
    """A /dev/shm that cannot hold the files (here: missing) sends them to the next directory; when no
    directory can, the other ranks build the BVH themselves instead of waiting (gloo, 2 ranks)."""
    import torch.multiprocessing as mp
    alt, out = tmp_path / "alt", tmp_path / "out"
    alt.mkdir()
    out.mkdir()
    mp.spawn(_share_worker, args=(2, bench._free_port(), str(tmp_path / "missing"), str(out), [str(alt)]),
             nprocs=2, join=True)
    assert (out / "r0").read_text() == "built|build"
    assert (out / "r1").read_text() == "True|adopt"
    assert list(alt.iterdir()) == []
    out2 = tmp_path / "out2"
    out2.mkdir()
    mp.spawn(_share_worker, args=(2, bench._free_port(), str(tmp_path / "missing"), str(out2),
                                  [str(tmp_path / "missing2")]), nprocs=2, join=True)
    assert (out2 / "r0").read_text() == "built|build"
    assert (out2 / "r1").read_text() == "built|build"
