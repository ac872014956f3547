"""Headline benchmark: Msamples/s of the HIP path tracer on the synthetic 10M-triangle soup
(BASELINE.json configs[2] / SURVEY.md §8d C3), 1920x1080, max_depth 5, tile-split across ranks.
The render form is the library's choice (the persistent path kernel on this scene);
config.form names it, and an untimed same-run leg reports north_star's wavefront layout beside it
(wavefront_ms_per_step).

A step is spp_per_step = ceil(--frame-spp / K) samples per pixel over the whole frame, so the K timed
steps render the metric's 1024-spp frame (--frame-spp, default 1024; the driver's --steps 20 renders
20 x 52 = 1040 spp).  The K steps are one render(spp = K * spp_per_step) call per rank over that rank's
tiles: a pixel's samples are one sequential chain through its sampler stream (cpu/integrator.cpp:
124-134), so the frame cannot be cut into independent per-step renders without repeating samples.
The frame-end gather to rank 0 (RCCL via torch.distributed) is inside the timed region.
value = W*H*K*spp_per_step / max-over-ranks time.

Launch: python bench.py [--gpus N --steps K --warmup W].  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank and --gpus must equal the world size.  Without it, --gpus N > 1 starts the N
ranks itself (a torch.distributed.run child, before anything touches the GPU) and fails loudly when
fewer than N devices are visible.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "akarirender-1_amd"))

METRIC = "Msamples/sec (whole node), 10M-tri scene 1080p 1024spp, 1/2/4/8 MI355X"
METRIC_CORNELL = "Msamples/sec, Cornell box 1080p 1024spp, 1x MI355X (BASELINE.json configs[1])"
METRIC_HALL = "Msamples/sec, Sponza-class textured scene 4K (BASELINE.json configs[3] stand-in), 1x MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate over the 8 XCDs
SCLK_HZ = 2.4e9                # MI355X shader clock (MI355X_MICROARCH.md: "120 cycles at 2.4 GHz")
RAY_BYTES, BOX_BYTES, TRI_BYTES = 32, 32, 40   # SURVEY.md §8d algorithmic bytes per ray / AABB / triangle test


TRACE_KERNEL_PROF_NAME = "k_trace<0, false, true, true>"   # closest hit, uncounted, tight cull, wide (rocprof name)
# persistent path kernel, uncounted (rocprof names: <COUNT, TAB> with the LDS scene tables since r13,
# <COUNT> before); the first one a profile holds is taken
PATH_KERNEL_PROF_NAME = ("k_path<false, true>", "k_path<false, false>", "k_path<false>")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def measured_traffic(kernel, workload, spp=None, profiles_dir=None):
    """The PMC record of `kernel` from the newest committed profile of this exact workload
    (profiles/<tag>_traffic.json, written by tools/prof_summary.py from separate rocprofv3 passes of
    tools/profile_driver.sh: read bytes from the fabric request counts by size, calibrated by
    tools/fetch_calib.hip, profiles/r21_fetch_calib.json).  A profile matches only when its
    workload equals the line's `config` field for field, so a 1-spp, unordered or whole-frame
    profile never stands in for a 1040-spp ordered launch or a rank's share.  PMC passes cannot run
    inside the timed region, so the figures are the profile's.  Returns (record, source) with
    `traffic` = HBM bytes of one launch (a persistent launch: per-spp bytes x `spp`), or (None, None)."""
    best = None
    names = [kernel] if isinstance(kernel, str) else list(kernel)
    for p in sorted(Path(profiles_dir or ROOT / "profiles").glob("*_traffic.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        w = d.get("workload") or {}
        name = next((k for k in names if k in d.get("kernels", {})), None)
        if name is None or any(w.get(k) != v for k, v in workload.items()) or set(w) - set(workload):
            continue
        rec = dict(d["kernels"][name])
        if spp is not None:   # a persistent launch renders every spp: scale the profile's per-spp bytes
            if "hbm_bytes_per_spp" not in rec:
                continue
            rec["traffic"] = rec["hbm_bytes_per_spp"] * spp
            if "read_bytes_per_spp" in rec:
                rec["read_traffic"] = rec["read_bytes_per_spp"] * spp
            if "l2_req_bytes_per_spp" in rec:
                rec["l2_bytes"] = rec["l2_req_bytes_per_spp"] * spp
        else:
            if "hbm_bytes_per_launch" not in rec:
                continue
            rec["traffic"] = rec["hbm_bytes_per_launch"]
            if "read_bytes" in rec:
                rec["read_traffic"] = rec["read_bytes"]
            if "l2_req_bytes_per_launch" in rec:
                rec["l2_bytes"] = rec["l2_req_bytes_per_launch"]
        best = (rec, f"profiles/{p.name}")
    return best if best else (None, None)


def latency_model(prof, cl, sh, npix, samples_per_s):
    """A ceiling for the latency-bound path kernel that does not saturate.
    Every ray is a chain of dependent fetches: the root box, one wide node per visit, one leaf
    record per leaf test (counted by the instrumented pass).  If each of the launch's resident lanes
    always had exactly one such fetch in flight and did nothing else, the launch would finish
    lanes / (rounds per sample x fetch latency) samples per second (Little's law), with the
    fetch latency the PMC pass's mean VMEM issue-to-return time (VmemLatency, cycles at SCLK_HZ).
    `frac` = achieved / that ceiling: the share of lane-time the chains actually spend waiting on
    their own next fetch.  It rises when lanes idle less (fuller waves, fewer processing phases) and
    falls when a change only shortens the latency the achieved rate is divided by."""
    c = prof.get("counters", {})
    lat = c.get("VmemLatency")
    lanes = prof.get("grid_threads")
    if not lat or not lanes:
        return None
    rounds = (cl["rays"] + cl["visits"] + cl["leaf_tests"] + sh["rays"] + sh["visits"] + sh["leaf_tests"]) / max(1, npix)
    lat_s = lat / SCLK_HZ
    ceiling = lanes / (rounds * lat_s)
    out = {"vmem_latency_cycles": round(lat, 1), "dependent_rounds_per_sample": round(rounds, 2),
           "resident_lanes": lanes, "ceiling_samples_per_s": round(ceiling, 1),
           "frac": round(samples_per_s / ceiling, 4)}
    if c.get("TCP_TCC_READ_REQ_sum"):
        out["l1_to_l2_read_latency_cycles"] = round(c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"], 1)
    if c.get("TCC_EA0_RDREQ_sum"):
        out["l2_to_fabric_read_latency_cycles"] = round(c["TCC_EA0_RDREQ_LEVEL_sum"] / c["TCC_EA0_RDREQ_sum"], 1)
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        out["wave_time"] = {"parked_waitcnt": round(c["SQ_WAIT_ANY"] / wc, 4),
                            "issue_stalled": round(c["SQ_WAIT_INST_ANY"] / wc, 4),
                            "issuing": round(c["SQ_ACTIVE_INST_ANY"] / wc, 4),
                            "valu_active": round(c["SQ_ACTIVE_INST_VALU"] / wc, 4)}
    return out


def time_split(pp, counts):
    """Where the persistent kernel's wave time goes, from the counting build's
    wave-uniform clocks over the untimed 1-spp counting pass (kernels.hip path_traverse / path_leaf):
    processing phases (shading among them), the traversal phase split into issuing the wide node's
    loads, waiting for them and the dependent work after them (slot tests, stack, ballots), the leaf
    phase split the same way (waiting for the header + two triangles; box and triangle tests), and the
    rest (loop control, the pixel fetch).  Fractions of the summed wave lifetimes; the lane factors
    (busy lanes per traversal slot, triangle tests per triangle-loop slot) say how much of a busy
    wave's issue does useful work."""
    tot = pp.get("t_total", 0)
    if not tot:
        return None
    f = lambda x: round(x / tot, 4)
    cl = counts["per_mode"]["closest"]
    sh = counts["per_mode"]["shadow"]
    out = {"processing": f(pp["t_proc"]), "shading": f(pp["t_shade"]),
           # k_path only (0 for the other forms): the processing phase's park, its sample end with the
           # splat / pixel fetch / camera ray, and the unpark with the new rays' start
           "processing_split": {"park": f(pp.get("tp_park", 0)), "results": f(pp["t_shade"]),
                                "results_record_load": f(pp.get("tp_load", 0)),
                                "sample_end_fetch_camera": f(pp.get("tp_next", 0)),
                                "unpark_ray_start": f(pp.get("tp_begin", 0))},
           "traversal": {"total": f(pp["t_trav"]), "issue": f(pp["tv_issue"]), "wait": f(pp["tv_wait"]),
                         "work": f(pp["tv_comp"])},
           "leaf": {"total": f(pp["t_leaf"]), "issue": f(pp["tl_issue"]), "wait": f(pp["tl_wait"]), "work": f(pp["tl_comp"])},
           "other": f(tot - pp["t_proc"] - pp["t_trav"] - pp["t_leaf"]),
           "lanes": {"traversal_busy": round((cl["visits"] + sh["visits"]) / max(1, cl["slots_traversal"]), 4),
                     "triangle_loop": round((cl["tri_tests"] + sh["tri_tests"]) / max(1, cl["slots_tri"]), 4),
                     # lanes holding a leaf when a wave enters its leaf phase (of 64), VERDICT r5 item 6
                     "leaf_phase_holders": round(pp.get("leaf_holders", 0) / max(1, pp.get("leaf_phases", 0)), 2)},
           "iterations_per_wave": round(pp["trav_iters"] / max(1, pp["waves"]), 1),
           # the launch lasts as long as its longest wave: the ratio to the mean wave is the launch's tail
           "longest_wave_over_mean": round(pp["t_max"] * pp["waves"] / tot, 4) if pp.get("waves") else None,
           "source": "counting build, untimed 1-spp pass; wave-uniform wall clocks (100 MHz) around an explicit "
                     "vmcnt(0) wait after each node / leaf load batch"}
    return out


from akari_amd.dist import tile_grid, tiles_for_rank, unpack_to_frame  # noqa: E402  (tile k -> rank k % world)


def host_cpus() -> dict:
    """The host's CPUs as the CPU baseline sees them: `nproc` (the affinity mask), os.cpu_count()
    (every online CPU, what std::thread::hardware_concurrency() reports), the cgroup CPU quota when
    one caps the job, and lscpu's model name.  `usable` = the CPUs this job can actually run on."""
    info = {"nproc": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count() or 1}
    usable = info["nproc"]
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            info["cgroup_cpus"] = round(int(quota) / int(period), 2)
            usable = max(1, min(usable, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                info["model"] = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    info["usable"] = usable
    return info


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_plan(gpus: int, env) -> tuple:
    """How this invocation runs: ("spawn", N) starts N ranks under torch.distributed.run;
    ("rank", world) runs as one rank of an already launched world (WORLD_SIZE in the environment,
    or a single process).  --gpus 0 means "whatever the launcher gave" (1 without one); a --gpus that
    contradicts a launcher's world size is an error, never a silently mislabelled line."""
    env_world = env.get("WORLD_SIZE")
    if env_world is None:
        if gpus > 1:
            return ("spawn", gpus)
        return ("rank", 1)
    world = int(env_world)
    if gpus and gpus != world:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return ("rank", world)


KFD_NODES = Path("/sys/class/kfd/kfd/topology/nodes")


def visible_gpu_count(env=None, kfd_nodes: Path = KFD_NODES) -> int:
    """GPUs this process may use, counted without torch or the HIP runtime (the launcher must not
    initialise the GPU before it starts the ranks: torch.cuda.device_count() can fall back to
    hipGetDeviceCount on this image).  KFD topology nodes with a non-zero gpu_id are the GPU agents;
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES narrow them as the runtime would.
    Each rank still checks its own device when it starts."""
    env = os.environ if env is None else env
    n = 0
    try:
        for node in kfd_nodes.iterdir():
            try:
                if int((node / "gpu_id").read_text().strip() or "0") != 0:
                    n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def spawn_ranks(n: int, argv, need_devices: bool = True) -> int:
    """Start n ranks of this script as a torch.distributed.run child (one process per GPU, RCCL
    over 127.0.0.1 rendezvous) and return its exit code.  Counts devices from sysfs first
    (visible_gpu_count): neither torch.cuda nor the HIP runtime is touched in this process, so the
    child start is never an exec after GPU initialisation."""
    if need_devices:
        have = visible_gpu_count()
        if have < n:
            raise SystemExit(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve()), *argv]
    log("[launcher] " + " ".join(cmd))
    return subprocess.run(cmd).returncode


def _bcast_from_rank0(obj):
    """Rank 0's `obj` on every rank (torch.distributed, the live group's backend)."""
    import torch.distributed as dist
    box = [obj]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def build_once_per_node(rank: int, build, export, adopt, barrier, tag: str, shm_dir: Path = Path("/dev/shm"),
                        fallback_dirs=None, bcast=None):
    """Rank 0 runs `build()` and leaves the BVH2 that `export()` returns in files (one .npy per array,
    written under a temporary name and renamed): in `shm_dir` when it has room, else in the first
    `fallback_dirs` entry that has (default: the temp dir; a container's /dev/shm may be 64 MB while
    the C3 BVH2 is 1.5 GB).  Rank 0 then broadcasts where the files are (`bcast`, default
    torch.distributed.broadcast_object_list), so a failed or impossible share never leaves a rank
    waiting: the other ranks map the files and run `adopt(nodes, tris)`, or run `build()` themselves
    when no directory had room, or raise when rank 0's build failed.  After a barrier rank 0 removes
    the files.  Returns what build / adopt returned."""
    bcast = bcast or _bcast_from_rank0
    dirs = [Path(shm_dir)] + [Path(d) for d in (fallback_dirs if fallback_dirs is not None
                                                 else [__import__("tempfile").gettempdir()])]
    names = ("nodes", "tris")
    files = lambda base: [Path(f"{base}_{n}{suf}.npy") for n in names for suf in ("", ".tmp")]
    info, where, err = None, None, None
    if rank == 0:
        try:
            info = build()
            nodes, tris = export()
            need = nodes.nbytes + tris.nbytes + (64 << 20)
            for d in dirs:
                base = d / f"akr_bench_bvh_{tag}"
                try:
                    if __import__("shutil").disk_usage(d).free < need:
                        log(f"[rank 0] BVH share: {d} has less than {need >> 20} MB free")
                        continue
                    for name, a in zip(names, (nodes, tris)):
                        tmp = Path(f"{base}_{name}.tmp.npy")
                        np.save(tmp, a)
                        os.replace(tmp, Path(f"{base}_{name}.npy"))
                    where = str(base)
                    break
                except OSError as e:
                    log(f"[rank 0] BVH share: {d} failed ({e})")
                    for f in files(base):
                        f.unlink(missing_ok=True)
            del nodes, tris
        except Exception as e:  # tell the other ranks before failing, so none waits for the files
            err = f"{type(e).__name__}: {e}"
            bcast({"where": None, "error": err})
            raise
    msg = bcast({"where": where, "error": err} if rank == 0 else None)
    if msg["error"]:
        raise RuntimeError(f"rank 0 failed to build the BVH: {msg['error']}")
    try:
        if rank != 0:
            if msg["where"]:
                base = msg["where"]
                info = adopt(np.load(f"{base}_nodes.npy", mmap_mode="r"), np.load(f"{base}_tris.npy", mmap_mode="r"))
            else:
                log(f"[rank {rank}] BVH share: no room to share, building locally")
                info = build()
        barrier()
    finally:  # the files hold ~1.5 GB of host memory: rank 0 removes them however the others fared
        if rank == 0 and where:
            for f in files(where):
                f.unlink(missing_ok=True)
    return info


def launch_check(world: int, rank: int):
    """--launch-check: the rank plumbing without a GPU (gloo): every rank joins the group and
    all-gathers a packed film the size of its tile share; rank 0 prints the live world size."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world and dist.get_rank() == rank
    film = torch.full((4 * 16,), float(rank))
    gathered = torch.empty(world * film.numel())
    if world > 1:
        dist.all_gather_into_tensor(gathered, film)
    else:
        gathered.copy_(film)
    ranks = sorted({int(v) for v in gathered.tolist()})
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_gathered": ranks}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# Untimed same-run legs of the other BASELINE configs: C2, the reference's Cornell
# box at 1920x1080 and 1024 spp, and the C4 stand-in (the synthetic textured hall) at 3840x2160 and
# 256 spp, each at its BASELINE spp in the library's form for that scene (~1.3 s and ~2.7 s).
SIDE_LEGS = {"cornell": (1920, 1080, 1024), "hall": (3840, 2160, 256)}


def side_leg(name, device, max_depth, tile, build_kw, stream_of):
    """Render one side configuration on `device` in a context of its own (scene, BVH, film) and time
    one render_device call of `spp` samples after a 1-spp warmup.  Returns the leg's record."""
    import torch
    from akari_amd import capi, scene
    W, H, spp = SIDE_LEGS[name]
    sc = (scene.cornell_scene(ROOT / "tests" / "golden" / "CornellBox-Original.obj.mesh", resolution=(W, H))
          if name == "cornell" else scene.hall_scene(resolution=(W, H)))
    cs = scene.compile_scene(sc)
    dev = torch.device("cuda", device)
    with capi.HipContext(device) as c:
        info = scene.upload_scene(c, cs, **build_kw)
        tiles = capi.rect_array(tile_grid(W, H, tile))
        film = torch.zeros(W * H * 4, device=dev)
        rad, wgt = film[:W * H * 3], film[W * H * 3:]
        st = stream_of(dev)
        c.render_device(1, max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), st)   # warm (pilot, kernels)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        c.render_device(spp, max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), st)
        torch.cuda.synchronize(dev)
        t = time.perf_counter() - t
        form = c.render_form()
        assert int(wgt.min().item()) == spp and int(wgt.max().item()) == spp
        return {"workload": {"cornell": "C2 Cornell box (BASELINE.json configs[1])",
                             "hall": "C4 stand-in: synthetic textured hall (BASELINE.json configs[3])"}[name],
                "triangles": cs.n_tris, "width": W, "height": H, "spp": spp, "max_depth": max_depth,
                "Msamples_per_s": round(W * H * spp / t / 1e6, 2), "ms_per_spp": round(t / spp * 1e3, 4),
                "form": form["form"], "ordered_fetch": form["ordered"], "bvh_nodes": info.n_nodes,
                "timed": False, "note": f"one render_device of {spp} spp after a 1-spp warmup, untimed leg of this run"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0,
                    help="ranks, one per GPU (0: the launcher's WORLD_SIZE, or 1); > 1 without a launcher "
                         "starts the ranks itself")
    ap.add_argument("--launch-check", action="store_true",
                    help="test the rank launch and the frame-end gather on CPU (gloo), no GPU work")
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps K; a step renders ceil(--frame-spp / K) spp of the whole frame")
    ap.add_argument("--warmup", type=int, default=2, help="untimed steps before the timed region (one render)")
    ap.add_argument("--frame-spp", type=int, default=1024,
                    help="spp the K timed steps render together at least (the metric's 1024-spp frame)")
    ap.add_argument("--scene", choices=["soup", "cornell", "hall"], default="soup",
                    help="soup: C3, the headline workload; cornell: C2 (BASELINE.json configs[1], the reference's "
                         "Cornell box at 1080p on one GPU); hall: C4 stand-in (configs[3], a synthetic textured hall "
                         "at 3840x2160); cornell and hall are side measurements, not the driver's line")
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--width", type=int, default=0, help="0: 1920 (3840 for --scene hall)")
    ap.add_argument("--height", type=int, default=0, help="0: 1080 (2160 for --scene hall)")
    ap.add_argument("--max-depth", type=int, default=5)
    # 64 x 64 tiles: interleaved over the ranks, a share's 64-pixel waves keep more spatial locality and
    # the ranks' costs even out better than with 32 x 32 (8-way share 0.798 / 0.798 against 0.808 /
    # 0.810 ms per spp, 4-way 1.365 against 1.391, whole frame unchanged; profiles/r20_tile_ab.log)
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--leaf", type=int, default=4)
    ap.add_argument("--bins", type=int, default=32, help="SAH bins per axis (reference: 32)")
    ap.add_argument("--sah-isect", type=float, default=4.0, help="SAH triangle-test cost (traversal step = 1)")
    ap.add_argument("--builder", choices=["sah", "lbvh", "sbvh"], default="sbvh",
                    help="host binned SAH, GPU LBVH, or host SBVH (the reference's spatial splits)")
    ap.add_argument("--spatial-budget", type=float, default=0.0,
                    help="SBVH: extra references allowed, as a fraction of the triangles (0: library default 0.5)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline workers (0: the host's hardware concurrency as this job sees it, "
                         "the reference's std::thread::hardware_concurrency(), core/parallel.cpp:32)")
    ap.add_argument("--cpu-frac", type=int, default=4, help="CPU sample = every n-th tile of the frame")
    ap.add_argument("--cpu-spp", type=int, default=1)
    ap.add_argument("--rays-per-lane", type=int, default=1, help="trace grid sizing (tuning)")
    ap.add_argument("--wide", type=int, default=1, help="4-wide quantized traversal (0: BVH2 kernel)")
    ap.add_argument("--lean", type=int, default=1, help="lean slot tests in the wide traversal (0: reference arithmetic)")
    ap.add_argument("--path", type=int, default=2,
                    help="1: the persistent path kernel (one launch per render); 0: the wavefront kernels; "
                         "2: the library's choice by the rank's pixel count (DESIGN.md §3.8)")
    ap.add_argument("--shadow-grid-pct", type=int, default=100, help="tuning: shadow-trace grid, %% of resident max")
    ap.add_argument("--timed-stats", type=int, default=-1,
                    help="HIP events inside the timed region: 2 = the dominant kernel (trace_closest) only, "
                         "1 = every kernel, 0 = none (probe), -1 = 1 on a whole frame, 2 on a share of a split")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="library option (akr_hip_set_option), repeatable; tuning / A-B only")
    ap.add_argument("--wavefront-spp", type=int, default=16,
                    help="untimed same-run leg in the wavefront form (north_star's layout), spp; 0 = skip")
    ap.add_argument("--count-lines", type=int, default=1,
                    help="1: an untimed 1-spp pass counting the distinct 128-B lines k_path reads (roofline.lines_per_pass)")
    ap.add_argument("--side-legs", type=int, default=1,
                    help="N = 1, soup: also render C2 (Cornell 1080p, 1024 spp) and the C4 stand-in (hall 4K, 256 spp) "
                         "as untimed legs of the same run (the line's `configs` block); 0 = skip")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="rehearse the N-rank path on a one-GPU box: every rank on device 0, a gloo process group, "
                         "the frame-end gather through host memory; the line says so and is not a measurement")
    ap.add_argument("--verify-frame", action="store_true",
                    help="N > 1: rank 0 assembles the gathered frame and checks it bit for bit against a single "
                         "whole-frame render of its own context (after the timed region; tests)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="single-process scaling probe: render only rank 0's tiles of an N-rank split "
                         "(prints the per-rank time; not a bench line for the driver)")
    args = ap.parse_args()

    how, world = launch_plan(args.gpus, os.environ)
    if how == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:], need_devices=not (args.launch_check or args.rehearse_one_gpu)))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        launch_check(world, rank)
        return

    import torch
    import torch.distributed as dist
    rehearse = args.rehearse_one_gpu and world > 1
    if rehearse:   # every rank on device 0; collectives on host tensors over gloo
        local = 0
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        if torch.cuda.device_count() <= local:
            raise SystemExit(f"bench.py: rank {rank} needs device {local}, {torch.cuda.device_count()} visible")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if world > 1:
        live = dist.get_world_size()   # n_gpus is the live group's size, never a flag
        if live != world:
            raise SystemExit(f"bench.py: launched for {world} ranks, process group has {live}")
        world = live
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if rehearse else dev   # where the collectives run

    from akari_amd import capi, scene

    W = args.width or (3840 if args.scene == "hall" else 1920)
    H = args.height or (2160 if args.scene == "hall" else 1080)
    K, Wm = args.steps, args.warmup
    if K < 1:
        raise SystemExit("bench.py: --steps must be >= 1")
    sps = max(1, -(-args.frame_spp // K))   # spp per step: K steps render >= --frame-spp spp
    spp = K * sps                           # the timed render's spp
    t0 = time.time()
    if args.scene == "cornell":
        sc = scene.cornell_scene(ROOT / "tests" / "golden" / "CornellBox-Original.obj.mesh", resolution=(W, H))
    elif args.scene == "hall":
        sc = scene.hall_scene(resolution=(W, H))
    else:
        sc = scene.soup_scene(n_tris=args.tris, resolution=(W, H))
    cs = scene.compile_scene(sc)
    t_gen = time.time() - t0
    ctx = capi.HipContext(local)
    t_setup = time.perf_counter()
    # host BVH build threads: the job's usable CPUs shared by the ranks of this node (16 at most)
    build_threads = max(2, min(16, host_cpus()["usable"] // max(1, world)))
    build_kw = dict(max_leaf_size=args.leaf, intersect_cost=args.sah_isect, n_bins=args.bins, n_threads=build_threads,
                    builder={"sah": capi.BUILDER_SAH, "lbvh": capi.BUILDER_LBVH, "sbvh": capi.BUILDER_SBVH}[args.builder],
                    spatial_budget=args.spatial_budget)
    if world > 1:
        # the node's ranks build the scene's BVH once (8 concurrent 10M-triangle SBVH builds would share
        # the host's CPUs): rank 0 builds it, the others adopt its BVH2 (akr_hip_import_accel:
        # validated, bit-identical results)
        full_kw = dict(build_kw, n_threads=max(2, min(16, host_cpus()["usable"])))
        info = build_once_per_node(
            rank, build=lambda: scene.upload_scene(ctx, cs, **full_kw), export=ctx.accel_export,
            adopt=lambda nodes, tris: scene.upload_scene(ctx, cs, bvh=(nodes, tris), n_threads=build_threads),
            barrier=dist.barrier, tag=os.environ.get("MASTER_PORT", "0"))
    else:
        info = scene.upload_scene(ctx, cs, **build_kw)
    t_setup = time.perf_counter() - t_setup  # BVH2 build (or import) + wide collapse + upload
    if args.rays_per_lane != 1:
        ctx.set_option("rays_per_lane", args.rays_per_lane)
    ctx.set_option("wide", args.wide)
    ctx.set_option("path", args.path)
    if not args.lean:
        ctx.set_option("lean", 0)
    if args.shadow_grid_pct != 100:
        ctx.set_option("shadow_grid_pct", args.shadow_grid_pct)
    for kv in args.opt:
        k, _, v = kv.partition("=")
        ctx.set_option(k, int(v))
    log(f"[rank {rank}] {args.scene} {cs.n_tris} tris gen {t_gen:.1f}s, BVH {info.n_nodes} nodes depth {info.max_depth} "
        f"build {info.build_ms / 1e3:.1f}s sah {info.sah_cost:.1f}")

    split = args.emulate_world if (args.emulate_world > 1 and world == 1) else world
    tiles = tiles_for_rank(W, H, args.tile, rank, split)
    npix = sum((x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in tiles)
    maxpix = max(sum((x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in tiles_for_rank(W, H, args.tile, r, split))
                 for r in range(split))
    tiles = capi.rect_array(tiles)   # the C-ABI's akr_rect array, made once (not inside the timed region)
    film = torch.zeros(maxpix * 4, device=dev)          # [radiance rgb (packed) | weight]
    rad, wgt = film[:maxpix * 3], film[maxpix * 3:]
    stream = torch.cuda.current_stream(dev).cuda_stream

    # warmup (also JIT/cache warm)
    if Wm > 0:
        ctx.render_device(Wm * sps, args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
    gathered = None
    if world > 1:
        # the frame-end gather once outside the timed region: RCCL connects a collective's channels
        # (ring peers over xGMI) on its first use, which must not land in the timed step
        gathered = torch.empty(world * film.numel(), device=cdev)
        dist.all_gather_into_tensor(gathered, film.to(cdev))
    torch.cuda.synchronize(dev)

    # untimed counting pass: traversal tests of one sample pass (algorithmic bytes)
    ctx.set_option("count_tests", 1)
    ctx.reset_stats()
    ctx.set_option("stats", 1)
    ctx.render_device(1, args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    counts = ctx.trace_counts()
    cstats = ctx.kernel_stats()
    pprof = ctx.path_profile()   # the counting build's phase clocks (persistent forms only)
    lines = None
    if pprof.get("waves") and args.count_lines and world == 1:
        # distinct 128-B lines one sample pass reads, in a pass of its own: k_path's
        # counting build marks every node / leaf / shading-record line in a bitmap (atomics: the clocks
        # of the pass above stay clean)
        ctx.set_option("count_lines", 1)
        ctx.render_device(1, args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        lp = ctx.path_profile()
        ctx.set_option("count_lines", 0)
        lines = {k: lp[f"lines_{k}"] for k in ("nodes", "leaves", "shading")}
    ctx.set_option("count_tests", 0)
    ctx.reset_stats()
    # events around every launch cost nothing on a whole frame but ~6 % of an 8-way rank's step;
    # trace_closest (the roofline kernel) is timed live either way
    timed_stats = args.timed_stats if args.timed_stats >= 0 else (1 if split == 1 else 2)
    ctx.set_option("stats", timed_stats)

    # timed region
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    ctx.render_device(spp, args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
    if world > 1:
        dist.all_gather_into_tensor(gathered, film.to(cdev))     # frame-end gather over RCCL
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    form = ctx.render_form()   # which form the library ran
    if world > 1:
        dist.barrier()
        tt = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    frame_check = None
    if args.verify_frame and world > 1:
        # the gathered films (the timed render's) assembled into the frame on rank 0 and compared
        # with one whole-frame render of rank 0's own context; every rank reports whether it adopted
        # rank 0's BVH (akr_hip_import_accel leaves build_ms 0) instead of building its own
        adopted = [None] * world
        dist.all_gather_object(adopted, bool(rank != 0 and info.build_ms == 0.0))
        if rank == 0:
            parts = gathered.cpu().numpy().reshape(world, -1)
            frad = np.zeros((H, W, 3), np.float32)
            fw = np.zeros((H, W), np.float32)
            for r in range(world):
                unpack_to_frame(parts[r], tiles_for_rank(W, H, args.tile, r, world), W, H, frad, fw)
            rrad, rw = ctx.render(spp, args.max_depth, tile_grid(W, H, args.tile), W, H)
            frame_check = {"bit_exact": bool(frad.tobytes() == rrad.tobytes() and fw.tobytes() == rw.tobytes()),
                           "max_abs_diff": float(np.abs(frad - rrad).max()), "weights_equal": bool(np.array_equal(fw, rw)),
                           "mean_radiance": float(rrad.mean() / max(1, spp)), "adopted_bvh": adopted,
                           "reference": "one whole-frame akr_hip_render of rank 0's context"}
    kstats = ctx.kernel_stats()
    passes = ctx.render_info()["passes"]
    # sanity: every pixel of this rank got every sample of the timed render
    assert int(wgt[:npix].min().item()) == spp and int(wgt[:npix].max().item()) == spp
    # untimed per-kernel breakdown (events on every launch) over a few more samples
    ctx.reset_stats()
    ctx.set_option("stats", 1)
    ctx.render_device(min(spp, 4), args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    bstats = ctx.kernel_stats()
    # wavefront form: the shadow trace timed alone (on the main stream, not overlapping the
    # closest-hit trace of the next bounce), for its own roofline
    iso = None
    if "trace_shadow" in bstats:
        ctx.reset_stats()
        ctx.set_option("serial_shadow", 1)
        ctx.render_device(min(spp, 4), args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        iso = ctx.kernel_stats()
        ctx.set_option("serial_shadow", 0)
    # untimed same-run leg in north_star's layout (wavefront: raygen -> closest -> shade -> shadow
    # -> splat launches per bounce), when the timed render ran a persistent kernel
    wavefront = None
    if rank == 0 and args.wavefront_spp > 0 and form["form"] in ("k_path", "k_path_defer", "k_path_spec"):
        # the wavefront, whatever form the timed render ran; the options in effect before are
        # restored afterwards
        saved = {k: ctx.option_set(k) for k in ("stats", "path")}
        ctx.reset_stats()
        ctx.set_option("stats", 0)
        ctx.set_option("path", 0)
        ctx.render_device(1, args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)   # warm
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        ctx.render_device(args.wavefront_spp, args.max_depth, tiles, rad.data_ptr(), wgt.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        tw = time.perf_counter() - tw
        wform = ctx.render_form()["form"]
        for k, v in saved.items():
            if v is not None:   # every one of them was set above (bench options / --opt)
                ctx.set_option(k, v)
        wavefront = {"ms_per_spp": round(tw / args.wavefront_spp * 1e3, 3), "spp": args.wavefront_spp,
                     "form": wform, "Msamples_per_s": round(npix * args.wavefront_spp / tw / 1e6, 3),
                     "timed": False}

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    if split != world:  # scaling probe: one rank's share of an N-way split, on this GPU
        print(json.dumps({"probe": "emulated rank 0 of a tile split", "emulate_world": split, "rank_pixels": npix,
                          "spp": spp, "rank_ms_per_spp": round(elapsed / spp * 1e3, 4),
                          "rank_Msamples_per_s": round(npix * spp / elapsed / 1e6, 3), "passes": passes,
                          "projected_node_Msamples_per_s": round(W * H * spp / elapsed / 1e6, 3),
                          "form": form, "wavefront": wavefront,
                          "kernels": {k: {"launches": v["launches"], "avg_ms": round(v["total_ms"] / v["launches"], 4)}
                                      for k, v in bstats.items()},
                          "rays_per_pixel": {"closest": counts["per_mode"]["closest"]["rays"] / max(1, npix),
                                             "shadow": counts["per_mode"]["shadow"]["rays"] / max(1, npix)}}),
              flush=True)
        return
    samples = W * H * spp
    value = samples / elapsed / 1e6
    config = {"workload": {"soup": "C3 synthetic triangle soup (SURVEY.md §8d)",
                           "cornell": "C2 Cornell box (reference fixture CornellBox-Original.obj.mesh, SURVEY.md §8d)",
                           "hall": "C4 stand-in: synthetic textured hall, Diffuse/Glossy/Mix with image textures, "
                                   "area lights (scene.hall_scene)"}[args.scene], "triangles": cs.n_tris,
              "width": W, "height": H, "spp_per_step": sps, "spp": spp, "max_depth": args.max_depth,
              "tile": args.tile, "parallelism": f"tile-split x{world}", "bvh_leaf": args.leaf,
              "sah_isect": args.sah_isect, "builder": args.builder,
              # the form the library ran (north_star names a wavefront; DESIGN.md §0 / §3.8 give the
              # measured reason for the persistent kernel on this scene) and the wavefront beside it
              "form": form["form"], "ordered_fetch": form["ordered"]}
    # roofline of the dominant kernel: the persistent path kernel (every closest-hit and shadow ray
    # of the render, SURVEY.md §8d "t_traversal_kernels"), or the wavefront's closest-hit trace
    cl = counts["per_mode"]["closest"]
    sh = counts["per_mode"]["shadow"]
    ray_bytes = lambda c: RAY_BYTES * c["rays"] + BOX_BYTES * c["box_tests"] + TRI_BYTES * c["tri_tests"]
    dom = "path" if "path" in cstats else "trace_closest"
    if dom == "path":   # the counting pass rendered 1 spp; the timed launch renders spp
        bytes_per_launch = (ray_bytes(cl) + ray_bytes(sh)) * spp
        prof_name = PATH_KERNEL_PROF_NAME
    else:
        bytes_per_launch = ray_bytes(cl) / (cstats.get("trace_closest", {}).get("launches", 0) or 1)
        prof_name = TRACE_KERNEL_PROF_NAME
    kc = kstats.get(dom) or bstats[dom]   # timed region (breakdown pass if --timed-stats 0)
    avg_ms = kc["total_ms"] / kc["launches"]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    # the PMC record of the same kernel from the committed profile of this exact config (the driver's
    # command, tools/profile_driver.sh); None when no profile of this config exists
    prof, traffic_src = measured_traffic(prof_name, config, spp=spp if dom == "path" else None)
    traffic = prof["traffic"] if prof else None
    # hardware fraction beside the model one: the PMC-measured HBM bytes over the live launch time
    hbm_achieved = traffic / (avg_ms * 1e-3) / 1e9 if traffic else None
    # read-only HBM fraction (north_star: "HBM-read roofline"): the L2 -> fabric read bytes, from the
    # request counts by size, calibrated on the traversal's widths (profiles/r21_fetch_calib.json: every
    # request is 128 B); Infinity-Cache hits are inside it, so it bounds the HBM reads from above
    read_traffic = prof.get("read_traffic") if prof else None
    hbm_read_achieved = read_traffic / (avg_ms * 1e-3) / 1e9 if read_traffic else None
    l2_bytes = prof.get("l2_bytes") if prof else None
    l2_achieved = l2_bytes / (avg_ms * 1e-3) / 1e9 if l2_bytes else None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "hbm_achieved": round(hbm_achieved, 1) if hbm_achieved else None,
                "hbm_frac": round(hbm_achieved / HBM_PEAK_GBS, 4) if hbm_achieved else None,
                "hbm_read_achieved": round(hbm_read_achieved, 1) if hbm_read_achieved else None,
                "hbm_read_frac": round(hbm_read_achieved / HBM_PEAK_GBS, 4) if hbm_read_achieved else None,
                "read_bytes_source": prof.get("read_bytes_source") if prof else None,
                "fetch_calibration": "profiles/r21_fetch_calib.json",
                # L2 request bandwidth of the same launch (TCC_REQ x 128 B, PMC) against the L2 peak
                "l2_achieved": round(l2_achieved, 1) if l2_achieved else None,
                "l2_peak": L2_PEAK_GBS,
                "l2_frac": round(l2_achieved / L2_PEAK_GBS, 4) if l2_achieved else None,
                "rays_per_sample": {"closest": cl["rays"] / max(1, npix), "shadow": sh["rays"] / max(1, npix)},
                "kernel": dom, "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_ms,
                "per_ray": {"box_tests": cl["box_tests"] / max(1, cl["rays"]),
                            "node_visits": cl["visits"] / max(1, cl["rays"]),
                            "leaf_tests": cl["leaf_tests"] / max(1, cl["rays"]),
                            "tri_tests": cl["tri_tests"] / max(1, cl["rays"])},
                "shadow_per_ray": {"box_tests": sh["box_tests"] / max(1, sh["rays"]),
                                   "node_visits": sh["visits"] / max(1, sh["rays"]),
                                   "leaf_tests": sh["leaf_tests"] / max(1, sh["rays"]),
                                   "tri_tests": sh["tri_tests"] / max(1, sh["rays"])},
                # SIMD lane utilisation of the traversal loop (node visits per lane slot) and of
                # the triangle loop (triangle tests per lane slot), from the counting pass; the path
                # kernel runs both ray kinds in one loop (its slots are counted with the closest set)
                "lane_util": ({"path": {"traversal": (cl["visits"] + sh["visits"]) / max(1, cl["slots_traversal"]),
                                        "holding_ray": cl["slots_busy"] / max(1, cl["slots_traversal"]),
                                        "triangles": (cl["tri_tests"] + sh["tri_tests"]) / max(1, cl["slots_tri"])}}
                              if dom == "path" else
                              {m: {"traversal": c["visits"] / max(1, c["slots_traversal"]),
                                   "holding_ray": c["slots_busy"] / max(1, c["slots_traversal"]),
                                   "triangles": c["tri_tests"] / max(1, c["slots_tri"])}
                               for m, c in (("closest", cl), ("shadow", sh))})}
    if dom == "path" and prof:
        roofline["latency"] = latency_model(prof, cl, sh, npix, value * 1e6)
    if dom == "path":
        roofline["time_split"] = time_split(pprof, counts)
    if lines:
        # the fabric's reads per sample pass against the distinct lines a pass touches: how often a line
        # is fetched again within a pass
        distinct = 128 * sum(lines.values())
        fabric = read_traffic / spp if (read_traffic and dom == "path") else None
        roofline["lines_per_pass"] = {**{k + "_gb": round(128 * v / 1e9, 4) for k, v in lines.items()},
                                      "distinct_gb": round(distinct / 1e9, 4),
                                      "fabric_read_gb": round(fabric / 1e9, 4) if fabric else None,
                                      "fabric_over_distinct": round(fabric / distinct, 2) if fabric and distinct else None,
                                      "source": "counting build, untimed 1-spp k_path pass, bitmap of 128-B lines"}
    if achieved > HBM_PEAK_GBS:   # the model bytes are not HBM bytes: caches serve most of them
        roofline["note"] = ("the SURVEY.md §8d algorithmic bytes exceed the HBM peak: most node and triangle reads "
                            "hit L2 or the Infinity Cache (on C3 ~66 % L2 hits by PMC, profiles/r20g_summary.md; a small scene's BVH is wholly "
                            "cache-resident), so frac is a model figure; hbm_frac is the HBM traffic measured by PMC "
                            "over the same launch time")
    if iso and "trace_shadow" in iso:   # the shadow trace alone: its own roofline (wavefront form)
        ks = iso["trace_shadow"]
        sms = ks["total_ms"] / ks["launches"]
        sb = ray_bytes(sh) / (cstats.get("trace_shadow", {}).get("launches", 0) or 1)
        roofline["shadow_isolated"] = {"kernel": "trace_shadow", "avg_launch_ms": sms, "bytes_per_launch": sb,
                                       "achieved": round(sb / (sms * 1e-3) / 1e9, 1),
                                       "frac": round(sb / (sms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                       "closest_isolated_ms": iso["trace_closest"]["total_ms"] / iso["trace_closest"]["launches"]}
    cpu = None
    if args.cpu_baseline and world == 1:
        sys.path.insert(0, str(ROOT / "oracle"))
        import py_oracle
        nodes, tris = ctx.accel_export()
        orc = py_oracle.OracleScene(cs, nodes, tris, capi)
        ctiles = tiles_for_rank(W, H, args.tile, 0, args.cpu_frac)
        cpx = sum((x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in ctiles)
        host = host_cpus()
        threads = args.cpu_threads or host["usable"]
        # the reference CPU path's traversal (exact intersectAABB), and the same port with the tight cull
        tc = time.perf_counter()
        orc.render(args.cpu_spp, args.max_depth, tiles=ctiles, n_threads=threads, exact_cull=True)
        dt = time.perf_counter() - tc
        tc = time.perf_counter()
        orc.render(args.cpu_spp, args.max_depth, tiles=ctiles, n_threads=threads, exact_cull=False)
        dt_tight = time.perf_counter() - tc
        cpu = {"value": round(cpx * args.cpu_spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads,
               "kind": "port", "host": host,
               "sample": f"every {args.cpu_frac}th {args.tile}x{args.tile} tile of the same frame ({cpx} px) x "
                         f"{args.cpu_spp} spp, same scene and BVH, reference intersectAABB, {dt:.1f} s",
               "value_tight_cull": round(cpx * args.cpu_spp / dt_tight / 1e6, 4)}

    configs = None
    if args.side_legs and world == 1 and args.scene == "soup":
        side_kw = dict(build_kw)
        configs = {}
        for name in SIDE_LEGS:
            try:   # a side leg never costs the headline line
                configs[name] = side_leg(name, local, args.max_depth, args.tile, side_kw,
                                         lambda d: torch.cuda.current_stream(d).cuda_stream)
            except Exception as e:  # noqa: BLE001  (reported in the line, not raised)
                configs[name] = {"error": f"{type(e).__name__}: {e}"}
            log(f"[rank 0] side leg {name}: {configs[name]}")

    line = {
        "metric": {"soup": METRIC, "cornell": METRIC_CORNELL, "hall": METRIC_HALL}[args.scene], "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": K, "warmup": Wm,
        "ms_per_step": round(elapsed / K * 1e3, 3), "ms_per_spp": round(elapsed / spp * 1e3, 4),
        "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic; REHEARSAL: the ranks shared one GPU and gathered over gloo, not a measurement"
                 if rehearse else "synthetic"),
        "config": config,
        "wavefront_ms_per_spp": wavefront["ms_per_spp"] if wavefront else None,
        "wavefront": wavefront,
        "roofline": roofline, "cpu_baseline": cpu, "frame_check": frame_check,
        "configs": configs,
        # per-kernel averages from an untimed pass with events on every launch (the timed region
        # times trace_closest only: events around every launch cost ~7 % at an 8-way rank)
        "kernels": {k: {"launches": v["launches"], "avg_ms": round(v["total_ms"] / v["launches"], 4)}
                    for k, v in bstats.items()},
        "bvh": {"nodes": info.n_nodes, "depth": info.max_depth, "build_s": round(info.build_ms / 1e3, 2),
                "setup_s": round(t_setup, 2), "build_threads": build_threads},
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
