#!/usr/bin/env python3
"""Benchmark: fingerprints/sec + match latency p50, 8 kHz mono (BASELINE.json:metric).

Step = one pass of the fingerprint hot path (create_audio_fingerprints, fp_handler.c:577-671)
over one batch of synthetic PCM already resident in HBM: configs[1] = 1,024 clips x 30 s at
8 kHz per GPU (960,512 fingerprints). Multi-GPU: one process per GPU (torchrun), each rank
fingerprints its own 1,024 clips (clip-sharded, no collective on the data path): weak scaling.

Also reported (same JSON line):
  roofline      the fingerprint kernel: algorithmic 520 B/fingerprint (512 B PCM in + 8 B out,
                SURVEY §8d) / average launch time measured with HIP events on the launch stream,
                against 8 TB/s HBM; traffic = PMC-measured HBM bytes per launch if a profile exists.
  strong        the same fixed 1,024-clip configs[1] batch split over the N ranks (strong scaling;
                north_star's >= 6x at 8 GPUs is graded on this leg's value at N = 1 vs 8).
  cpu_baseline  the C oracle (oracle/, the reference path restated; `port`) on a bounded sample of
                the same workload: the host's CPU share (16 threads on a 1-GPU box; `nproc`
                reported beside it) and 1 thread.
  match         configs[2]: 4,096 x 5 s queries vs a 100k-clip DB (93.8 M rows), coefs=1,
                tolerance 0.001; batch-4096 time and batch-1 latency p50/p99 (host PCM in ->
                result out); with N GPUs the DB is clip-sharded and the per-query keys are
                combined by one RCCL all_reduce(MAX) (configs[3]).
  stream        configs[4]: 512 live channels, 160-sample ticks, 3 s window, matched every tick;
                with N GPUs the channels are split over the ranks against a replicated DB.
  group         the in-process device group (tfp_group_*): the path the Asterisk shim serves its
                channel threads with (one process, one handle, fp_handler.c:1161-1169), over every
                GPU the process sees: the configs[3] batch from host PCM, batch-1 latency and the
                512-channel stream through the same entry points the shim calls.

--gpus N: under a launcher (torchrun / torch.distributed.run: WORLD_SIZE set) WORLD_SIZE must equal
N, or bench.py exits non-zero; without one, bench.py starts the N rank processes itself (a child
torch.distributed.run, before any GPU call) and exits with its code. It never runs fewer ranks than
asked.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "asterisk-tiresias_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

HOP = 256
BYTES_PER_FP = 512 + 8
HBM_PEAK_GBS = 8000.0
SEED_DB, SEED_Q = 0x7153A1, 0x7153B2


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def uuid_of(global_clip: int) -> str:
    """Deterministic v4-shaped uuid per global clip id (same on every rank)."""
    a = (global_clip * 0x9E3779B97F4A7C15 + 0x7153A1) & (2**64 - 1)
    b = (a * 0xBF58476D1CE4E5B9 + global_clip) & (2**64 - 1)
    x = (a << 64) | b
    s = "%032x" % x
    s = s[:12] + "4" + s[13:16] + "89ab"[int(s[16], 16) & 3] + s[17:]
    return "%s-%s-%s-%s-%s" % (s[:8], s[8:12], s[12:16], s[16:20], s[20:32])


def launch_plan(gpus: int, env, argv):
    """How this process runs `--gpus gpus`: ("run", None) when it is one rank of a launcher's job
    (WORLD_SIZE == gpus) or gpus == 1 without one; ("spawn", cmd) without a launcher for gpus > 1:
    cmd starts the gpus rank processes (torch.distributed.run, rendezvous on 127.0.0.1) with the
    same arguments; ("refuse", why) when a launcher's WORLD_SIZE disagrees with --gpus."""
    ws = env.get("WORLD_SIZE")
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: need at least 1"
    if ws is not None:
        if int(ws) != gpus:
            return "refuse", f"--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks"
        return "run", None
    if gpus == 1:
        return "run", None
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    return "spawn", [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
                     "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


# Fields the device-group leg reports besides its timings (an N-GPU line shows which devices the
# group spanned and whether xGMI peer access came up for every ordered pair of them).
GROUP_FIELDS = ("n_devices", "devices", "peer_access", "shards_rows_clips", "equal_to_engine")


def dist_report(dist, rank, world, backend, device):
    """The world size every rank's process group reports, gathered on every rank (the bench line's
    `dist`); a rank that disagrees stops the run."""
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "world_size": dist.get_world_size(), "device": device})
    rep = {"backend": backend + (" (RCCL)" if backend == "nccl" else ""), "ranks": seen,
           "all_ranks_saw_world": all(x["world_size"] == world for x in seen)}
    if not rep["all_ranks_saw_world"]:
        raise SystemExit(f"ranks disagree on the world size: {seen}")
    return rep


def launch_check(args):
    """--launch-check (tests/test_bench_launch.py): the ranks meet over gloo and rank 0 prints the
    world size it sees and every rank's report of it (the `dist` field of the bench line), with no
    GPU call at all."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n = world
    rep = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        n = int(t.item())
        rep = dist_report(dist, rank, world, "gloo", int(os.environ.get("LOCAL_RANK", "0")))
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"launch_check": True, "gpus": args.gpus, "world_size": world, "ranks_met": n, "dist": rep,
                          "group_fields": list(GROUP_FIELDS)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=1024)
    ap.add_argument("--seconds", type=int, default=30)
    ap.add_argument("--db-clips", type=int, default=100_000)
    ap.add_argument("--queries", type=int, default=4096)
    ap.add_argument("--latency-queries", type=int, default=40)
    ap.add_argument("--no-match", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-db-clips", type=int, default=1000,
                    help="30 s clips in the SQLite DB of the match CPU baseline")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling leg")
    ap.add_argument("--no-sweeps", action="store_true", help="skip the match leg's tolerance / coefs sweeps")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1),
                    help="host threads of the full-DB CPU comparison (16 = the GPU box's CPU share)")
    ap.add_argument("--no-enrol", action="store_true", help="skip the enrol-then-first-search latency")
    ap.add_argument("--clock-warmup-s", type=float, default=0.25,
                    help="untimed fingerprint steps before the timed region until this much wall time has passed")
    ap.add_argument("--stream-channels", type=int, default=512)
    ap.add_argument("--stream-ticks", type=int, default=200)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on MI355X; gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--no-group", action="store_true", help="skip the in-process device-group leg")
    ap.add_argument("--launch-check", action="store_true", help="start the ranks, meet over gloo, print, exit (no GPU)")
    args = ap.parse_args()

    # --gpus N: every rank process exists before any GPU call (a child launcher, never an exec)
    how, what = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if how == "refuse":
        log(f"bench.py: {what}")
        sys.exit(2)
    if how == "spawn":
        log(f"bench.py: starting {args.gpus} ranks: {' '.join(what)}")
        sys.exit(subprocess.call(what))
    if args.launch_check:
        launch_check(args)
        return

    import torch
    import tiresias_amd as T

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ndev = torch.cuda.device_count()
    gpu = local if args.dist_backend == "nccl" else local % max(ndev, 1)
    torch.cuda.set_device(gpu)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", gpu)
    # the world size every rank's process group reports (an 8-GPU line shows all eight met)
    dist_info = dist_report(dist, rank, world, args.dist_backend, gpu) if dist else None
    eng = T.Engine(gpu)
    # a real (non-null) stream: every launch and every event goes on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    assert sh, "need a non-default stream handle"

    def barrier():
        if dist:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if not dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---------------------------------------------------------------- fingerprint (C2)
    n = 8000 * args.seconds
    nclips = args.clips
    pcm = torch.empty((nclips, n), dtype=torch.int16, device=dev)
    eng.synth_device(SEED_DB, range(rank * nclips, (rank + 1) * nclips), n, pcm.data_ptr(), stream=sh)
    offsets = np.arange(nclips + 1, dtype=np.int64) * n
    plan = eng.plan(offsets)
    F = plan.nframes
    micro = torch.empty((F, 2), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, sh)
    torch.cuda.synchronize(dev)
    # Clock warm-up (untimed): the GPU ramps its clock over tens of ms of load, so a few warmup
    # steps leave the timed steps partly at a lower clock (0.60 vs 0.54 ms per C2 step measured
    # with 3 vs 50 warmup steps). Keep stepping until >= --clock-warmup-s of wall time.
    t_w = time.perf_counter()
    n_clock = 0
    while time.perf_counter() - t_w < args.clock_warmup_s:
        for _ in range(16):
            eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, sh)
        torch.cuda.synchronize(dev)
        n_clock += 16
    barrier()
    torch.cuda.synchronize(dev)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, sh)
        evs[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    launch_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    wall = max_over_ranks(wall)
    ms_step = wall * 1e3 / args.steps
    total_fp = F * world * args.steps
    value = total_fp / wall
    avg_launch_s = float(np.mean(launch_ms)) / 1e3
    achieved = BYTES_PER_FP * F / avg_launch_s / 1e9
    traffic = None
    tpath = os.path.join(REPO, "profiles", "traffic_fingerprint.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("frames_per_launch") == F:
            traffic = tj.get("hbm_bytes_per_launch")
    issue = None
    ipath = os.path.join(REPO, "profiles", "issue_fingerprint.json")
    if os.path.exists(ipath):
        with open(ipath) as f:
            ij = json.load(f)
        if ij.get("frames_per_launch") == F:
            valu_s = ij["valu_per_frame"] * F / avg_launch_s
            issue = {"bound": "valu_issue", "achieved": valu_s, "peak": ij["valu_issue_peak_per_s"],
                     "unit": "wave64 VALU instructions/s", "frac": valu_s / ij["valu_issue_peak_per_s"],
                     "valu_per_unit": ij["valu_per_frame"], "lds_per_unit": ij["lds_per_frame"],
                     "wave_cycle_split": ij["wave_cycle_split"], "peak_method": ij["peak_method"],
                     "counts_from": ij["source"]}
    log(f"[rank {rank}] fingerprint: {F} fp/launch, avg launch {avg_launch_s*1e3:.3f} ms, {F/avg_launch_s/1e9:.3f} Gfp/s")

    out = {
        "metric": "fingerprints/sec + match latency p50, 8 kHz mono, 1/2/4/8 MI355X",
        "value": value,
        "unit": "fingerprints/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "clock_warmup_steps": n_clock,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (deterministic counter-based 8 kHz PCM, tfp_synth)",
        "config": {"workload": f"configs[1]: {nclips} x {args.seconds} s 8 kHz mono clips per GPU, fingerprint-only",
                   "clips_per_gpu": nclips, "samples_per_clip": n, "frames_per_step_per_gpu": F,
                   "parallelism": f"clip-sharded x{world}"},
        "roofline": {"bound": "hbm", "kernel": "fingerprint8k_kernel + finish_db_kernel", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "bytes_per_unit": BYTES_PER_FP, "units_per_launch": F, "avg_launch_ms": avg_launch_s * 1e3,
                     "limiter": "not HBM: per-wave issue and latency at 2 waves/SIMD (~170 wave64 VALU + ~24 LDS + ~13 SALU "
                                "per fingerprint; bit-exact fp32 DSP + glibc-exact logs); see `issue` and DESIGN.md §4",
                     "issue": issue},
        # the same throughput as clips/s and as multiples of real time (a fingerprint
        # is one 256-sample hop of 8 kHz audio)
        "derived": {"clips_per_s": value * nclips / (F or 1), "x_realtime": value * HOP / 8000.0,
                    "clip_seconds": n / 8000.0},
    }
    if dist_info:
        out["dist"] = dist_info
    del micro

    # ---------------------------------------------------------------- strong scaling (C2 fixed)
    if not args.no_strong:
        out["strong"] = run_strong(args, eng, torch, dev, sh, pcm, nclips, n, rank, world, barrier, max_over_ranks)

    # ---------------------------------------------------------------- CPU baseline (oracle)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = fingerprint_cpu_baseline(args, pcm, nclips, n, F)
    del pcm
    torch.cuda.empty_cache()

    # ---------------------------------------------------------------- match (C3 / C4)
    if not args.no_match and args.db_clips > 0:
        out["match"] = run_match(args, eng, torch, dev, sh, rank, world, dist, barrier, max_over_ranks, T)
        if args.stream_channels > 0:
            out["stream"] = run_stream(args, eng, T, torch, dev, sh, rank, world, dist, barrier)
        if not args.no_group:
            out["group"] = run_group(args, eng, T, torch, dev, sh, rank, world, dist)

    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def run_strong(args, eng, torch, dev, sh, pcm, nclips, n, rank, world, barrier, max_over_ranks):
    """Strong scaling: the fixed configs[1] batch (nclips clips in total, not per GPU) split over
    the ranks in contiguous shares; each rank times K launches over its share (taken from the
    weak leg's PCM, already in HBM), wall time max over ranks, value = the batch's frames per
    second. At N = 1 this is the weak leg's workload, timed again."""
    share = [(nclips * r) // world for r in range(world + 1)]
    b, e = share[rank], share[rank + 1]
    k = e - b
    plan = eng.plan(np.arange(k + 1, dtype=np.int64) * n)
    micro = torch.empty((max(plan.nframes, 1), 2), dtype=torch.int32, device=dev)
    d_pcm = pcm[b:e].data_ptr() if k else pcm.data_ptr()

    def step():
        if k:
            eng.fingerprint_device(plan, d_pcm, micro.data_ptr(), 0, sh)
    for _ in range(max(args.warmup, 3)):
        step()
    torch.cuda.synchronize(dev)
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < args.clock_warmup_s:  # clock warm-up, as for the weak leg
        for _ in range(16):
            step()
        torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    wall = max_over_ranks(time.perf_counter() - t0)
    total = nclips * ((n + HOP - 1) // HOP)
    log(f"[rank {rank}] strong: {k} of {nclips} clips, {wall * 1e3 / args.steps:.3f} ms per step (max over ranks)")
    res = {"workload": f"configs[1] fixed: {nclips} x {args.seconds} s clips in total, split over {world} GPU(s)",
           "scaling": "strong", "clips_total": nclips, "clips_per_gpu_max": max(share[r + 1] - share[r] for r in range(world)),
           "frames_per_step": total, "ms_per_step": wall * 1e3 / args.steps, "value": total * args.steps / wall,
           "unit": "fingerprints/s"}
    if world == 1:
        res["projected"] = strong_projection(args, eng, torch, dev, sh, pcm, nclips, n, wall / args.steps)
    return res


def strong_projection(args, eng, torch, dev, sh, pcm, nclips, n, t_full):
    """One GPU's share of the fixed batch at N = 2, 4, 8 (1,024 / N clips), timed on this GPU with
    HIP events over K launches: the strong leg's per-rank work, so t(1,024 clips) / t(share) is the
    speedup N GPUs can reach before collectives and launch skew (the fingerprint leg has none)."""
    out = {}
    for N in (2, 4, 8):
        k = nclips // N
        plan = eng.plan(np.arange(k + 1, dtype=np.int64) * n)
        micro = torch.empty((max(plan.nframes, 1), 2), dtype=torch.int32, device=dev)
        for _ in range(3):
            eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, sh)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < args.clock_warmup_s:
            for _ in range(16):
                eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, sh)
            torch.cuda.synchronize(dev)
        reps = max(args.steps, 20)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            eng.fingerprint_device(plan, pcm.data_ptr(), micro.data_ptr(), 0, sh)
        e1.record()
        torch.cuda.synchronize(dev)
        t_share = e0.elapsed_time(e1) / 1e3 / reps
        out[str(N)] = {"clips_per_gpu": k, "ms_per_step": t_share * 1e3, "projected_speedup": t_full / t_share,
                       "projected_efficiency": t_full / t_share / N}
        log(f"strong projection N={N}: {k} clips {t_share * 1e3:.3f} ms -> x{t_full / t_share:.2f}")
        del micro
    return out


def fingerprint_cpu_baseline(args, pcm, nclips, n, F):
    """The C oracle (the reference's create_audio_fingerprints restated, `port`: libaubio is not
    in the image) on whole passes over a sample of the batch's clips, on the host's CPU share and
    on one thread."""
    import oracle_py
    nproc = os.cpu_count() or 1
    # the GPU box's CPU share (OMP_NUM_THREADS, 16 per GPU there); nproc counts the whole machine
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or nproc
    threads = max(1, min(nproc, share))
    k = min(nclips, 4 * threads)
    host = pcm[:k].cpu().numpy().reshape(-1)
    off = np.arange(k + 1) * n
    oracle_py.fingerprint_batch(host[: 2 * n], off[:3], nthreads=1, want_db=False)  # load + tables

    def timed(nthreads, clips, seconds):
        passes, t1 = 0, time.perf_counter()
        while True:  # whole passes over the sample until ~seconds of work
            oracle_py.fingerprint_batch(host[: clips * n], off[: clips + 1], nthreads=nthreads, want_db=False)
            passes += 1
            dt = time.perf_counter() - t1
            if dt >= seconds:
                return passes, dt
    passes, dt = timed(threads, k, args.cpu_seconds)
    frames = passes * k * (F // nclips)
    fps = frames / dt
    p1, dt1 = timed(1, 2, max(2.0, args.cpu_seconds / 3))
    fps1 = p1 * 2 * (F // nclips) / dt1
    # every core the machine reports (nproc), beside the share: on a shared GPU box the extra
    # threads compete for the share's cores, so this is the figure for a dedicated host
    ka = min(nclips, max(k, nproc))
    host_all = pcm[:ka].cpu().numpy().reshape(-1) if ka > k else host
    off_all = np.arange(ka + 1) * n
    pa, ta = 0, time.perf_counter()
    while True:
        oracle_py.fingerprint_batch(host_all[: ka * n], off_all, nthreads=nproc, want_db=False)
        pa += 1
        dta = time.perf_counter() - ta
        if dta >= max(2.0, args.cpu_seconds / 2):
            break
    fpsa = pa * ka * (F // nclips) / dta
    log(f"cpu baseline {fps:.0f} fp/s on {threads} threads ({dt:.1f} s), {fps1:.0f} fp/s on 1 thread, "
        f"{fpsa:.0f} fp/s on {nproc} threads; nproc {nproc}")
    return {"value": fps, "unit": "fingerprints/s", "cores": threads, "kind": "port",
            "sample": f"{passes} passes over {k} of the {nclips} x {args.seconds} s clips "
                      f"({frames} frames), oracle/oracle.c, {threads} threads, {dt:.1f} s",
            "nproc": nproc, "cores_policy": "the host's CPU share for this GPU (OMP_NUM_THREADS; 16 per GPU on "
                                            "the GPU box), capped at nproc",
            "one_core": {"value": fps1, "unit": "fingerprints/s", "cores": 1,
                         "sample": f"{p1} passes over 2 clips ({p1 * 2 * (F // nclips)} frames), 1 thread, {dt1:.1f} s"},
            "all_cores": {"value": fpsa, "unit": "fingerprints/s", "cores": nproc,
                          "sample": f"{pa} passes over {ka} clips ({pa * ka * (F // nclips)} frames), {nproc} threads "
                                    f"(nproc), {dta:.1f} s"},
            "note": "libaubio is not installed: the oracle restates its algorithm in plain C (kind: port)"}


def enroll(eng, torch, dev, sh, ids_all, chunk=2048):
    """Clear the index and enrol the synthetic 30 s DB clips `ids_all` (synthesised, fingerprinted
    and added on the device, 2048 clips at a time)."""
    n_db = 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    buf = torch.empty((chunk, n_db), dtype=torch.int16, device=dev)
    micro = torch.empty((chunk * nf_db, 2), dtype=torch.int32, device=dev)
    plan = eng.plan(np.arange(chunk + 1, dtype=np.int64) * n_db)
    eng.index_clear()
    for s in range(0, len(ids_all), chunk):
        ids = ids_all[s:s + chunk]
        k = len(ids)
        if k < chunk:
            plan = eng.plan(np.arange(k + 1, dtype=np.int64) * n_db)
        eng.synth_device(SEED_DB, ids, n_db, buf.data_ptr(), stream=sh)
        eng.fingerprint_device(plan, buf.data_ptr(), micro.data_ptr(), 0, sh)
        eng.index_add_device([uuid_of(g) for g in ids], np.arange(k + 1, dtype=np.int64) * nf_db, micro.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    del buf, micro
    torch.cuda.empty_cache()


def c3_queries(eng, torch, dev, sh, nq, db_clips, qn=8000 * 5):
    """configs[2]'s query batch on the device, int16 [nq, qn]: 75 % excerpts of DB clips at
    256-aligned offsets, 25 % unrelated audio (the same on every rank; tests reuse it)."""
    n_db = 8000 * 30
    rng = np.random.default_rng(SEED_Q)
    seeds, clips, offs = [], [], []
    for i in range(nq):
        if i % 4 != 3:
            clips.append(int(rng.integers(db_clips)))
            offs.append(256 * int(rng.integers(0, (n_db - qn) // HOP)))
            seeds.append(SEED_DB)
        else:
            clips.append(i)
            offs.append(0)
            seeds.append(SEED_Q)
    qpcm = torch.empty((nq, qn), dtype=torch.int16, device=dev)
    for sd in (SEED_DB, SEED_Q):
        idx = [i for i in range(nq) if seeds[i] == sd]
        tmp = torch.empty((len(idx), qn), dtype=torch.int16, device=dev)
        eng.synth_device(sd, [clips[i] for i in idx], qn, tmp.data_ptr(), offsets=[offs[i] for i in idx], stream=sh)
        qpcm[torch.tensor(idx, device=dev)] = tmp
    torch.cuda.synchronize(dev)
    return qpcm


def run_match(args, eng, torch, dev, sh, rank, world, dist, barrier, max_over_ranks, T):
    from tiresias_amd import sharding
    n_db = 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    from tiresias_amd import sharding
    mine = sharding.shard_clips(args.db_clips, world, rank).tolist()  # clip-sharded round robin
    t_build = time.perf_counter()
    enroll(eng, torch, dev, sh, mine)
    # global tie-break: rank of each uuid among all clips (every rank derives it, no exchange)
    if world > 1:
        grank = sharding.global_tiebreak([uuid_of(g) for g in range(args.db_clips)])
        eng.set_tiebreak(grank[mine])
    eng.index_commit()
    torch.cuda.synchronize(dev)
    t_build = time.perf_counter() - t_build
    rows, nclips_local = eng.index_stats()

    nq, qn = args.queries, 8000 * 5
    qpcm = c3_queries(eng, torch, dev, sh, nq, args.db_clips)
    qplan = eng.plan(np.arange(nq + 1, dtype=np.int64) * qn)
    keys = torch.zeros(nq, dtype=torch.int64, device=dev)
    p = T.params(1, 0.001)
    # N ranks: each fingerprints 1/N of the queries, all_gather of their frame values, search of
    # the local clips, all_reduce(MAX) of the keys (sharding.QueryShardedSearch); 1 rank: one call
    sharded = sharding.QueryShardedSearch(eng, torch, dev, dist, nq, qn) if world > 1 and nq % world == 0 else None

    def batch():
        if sharded:
            sharded(qpcm.data_ptr(), p, keys, sh)
        else:
            eng.search_device(qplan, qpcm.data_ptr(), p, keys.data_ptr(), sh)
            sharding.combine(keys, dist)
    torch.cuda.synchronize(dev)
    # untimed: 2 calls, then back-to-back calls for --clock-warmup-s so the batches are timed at
    # the steady-state clock, as the fingerprint steps are
    # (a count every rank agrees on: with N ranks each batch holds collectives)
    batch()
    batch()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    batch()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter() - t1
    n_more = int(max_over_ranks(float(math.ceil(args.clock_warmup_s / max(t1, 1e-5)))))
    for _ in range(n_more):
        batch()
    n_warm = 3 + n_more
    torch.cuda.synchronize(dev)
    reps = 5
    times = []
    for _ in range(reps):
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        batch()
        torch.cuda.synchronize(dev)
        times.append(max_over_ranks(time.perf_counter() - t0))
    batch_ms = float(np.median(times)) * 1e3
    k = keys.cpu().numpy().view(np.uint64)
    found = int((k != 0).sum())

    # SURVEY §8(d) sweeps on the same batch: tolerances, coefs = 2 (the general path), and the
    # 100 / 3400 Hz ignore filter — which drops ~92% of the synthetic frames (their max1 sits at
    # 16.8-17.2 dB, under 10*log10(100) = 20 dB) and so finds nothing — plus 50 / 60 Hz
    # (16.99 / 17.78 dB), which keeps about a third of them. First call untimed (it builds the tolerance's caches), then
    # the median of up to 5 timed calls (1 when a call takes over 2 s).
    sweeps = []
    if not args.no_sweeps:
        for coefs, tol, low, high in [(1, 0.01, -1, -1), (1, 0.1, -1, -1), (1, 0.45, -1, -1), (1, 0.001, 100, 3400),
                                      (1, 0.001, 50, 60), (2, 0.001, -1, -1), (2, 0.01, -1, -1), (2, 0.1, -1, -1),
                                      (2, 0.45, -1, -1), (2, 0.1, 100, 3400), (2, 0.01, 50, 60)]:
            ps = T.params(coefs, tol, low, high)
            log(f"sweep coefs={coefs} tol={tol} low/high={low}/{high} ...")

            def sweep_batch():
                if sharded:
                    sharded(qpcm.data_ptr(), ps, keys, sh)
                else:
                    eng.search_device(qplan, qpcm.data_ptr(), ps, keys.data_ptr(), sh)
                    sharding.combine(keys, dist)
            sweep_batch()
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(5):
                barrier()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                sweep_batch()
                torch.cuda.synchronize(dev)
                ts.append(max_over_ranks(time.perf_counter() - t0))
                if ts[-1] > 2.0:
                    break
            ks = keys.cpu().numpy().view(np.uint64)
            sweeps.append({"coefs": coefs, "tolerance": tol, "freq_ignore_low": low, "freq_ignore_high": high,
                           "batch_ms": float(np.median(ts)) * 1e3, "queries_per_s": nq / float(np.median(ts)),
                           "found": int((ks != 0).sum()), "timed_calls": len(ts)})
            log(f"sweep coefs={coefs} tol={tol} low/high={low}/{high}: {sweeps[-1]['batch_ms']:.2f} ms, "
                f"found {sweeps[-1]['found']}")

    # batch-1 latency: host PCM in -> (uuid, match_count, frame_count) out
    # On N GPUs every rank runs the same small-batch path on its shard, turns its local winner into
    # the global key (match_count << 32 | global uuid rank) and one all_reduce(MAX) of 8 bytes
    # picks the winner with the reference's tie-break.
    host_q = qpcm[: args.latency_queries].cpu().numpy()
    if dist:
        uuid_grank = {uuid_of(g): int(grank[g]) for g in range(args.db_clips)}
        kpin = torch.zeros(1, dtype=torch.int64).pin_memory()
        kdev = torch.zeros(1, dtype=torch.int64, device=dev)
    for i in range(min(3, len(host_q))):  # untimed: first-call allocations of the small path
        eng.search_pcm_batch(host_q[i], [0, qn], p)
    lat = []
    for i in range(len(host_q)):
        barrier()
        t0 = time.perf_counter()
        res, _ = eng.search_pcm_batch(host_q[i], [0, qn], p)
        if dist:
            r = res[0]
            kpin[0] = sharding.make_key(r["match_count"], uuid_grank[r["audio_uuid"]]) if r else 0
            kdev.copy_(kpin, non_blocking=True)
            sharding.combine(kdev, dist)
            kdev.item()
        lat.append(max_over_ranks(time.perf_counter() - t0) * 1e3)
    lat_py = list(lat)
    threads = None
    harness = "python (ctypes) loop, max over ranks + 8-byte all_reduce" if dist else "python (ctypes) loop"
    if not dist:
        # the same calls from C (asterisk-tiresias_amd/bench/tfp_latency.c), as the Asterisk shim's
        # channel threads make them: no Python/ctypes marshalling in the timed region
        clat = ctypes.CDLL(os.path.join(os.path.dirname(T.LIB_PATH), "libtfp_latency.so"))
        n_it = max(200, 10 * len(host_q))
        out_ms = np.zeros(n_it, np.float64)
        fnd = np.zeros(n_it, np.int32)
        hq = np.ascontiguousarray(host_q, np.int16)
        rc = clat.tfp_latency_search_pcm(eng.handle, ctypes.c_void_p(hq.ctypes.data), ctypes.c_int64(qn),
                                         ctypes.c_int32(len(hq)), ctypes.c_int32(8000), ctypes.byref(p),
                                         ctypes.c_int32(n_it), ctypes.c_void_p(out_ms.ctypes.data),
                                         ctypes.c_void_p(fnd.ctypes.data))
        if rc == 0:
            lat = out_ms.tolist()
            harness = ("C loop over tfp_search_pcm_batch (bench/tfp_latency.c), %d calls over %d queries held in a "
                       "tfp_host_alloc buffer (read in place, as the shim's WAV reads)" % (n_it, len(hq)))
        threads = concurrent_searches(eng, T, clat, hq, qn, p)
    # SURVEY §8(d)'s match roofline: one pass over the index per batch (12 B per row) plus the
    # query frames (16 B each) against HBM; the vote path reads only the used keys' boxes, so a
    # fraction above 1 means the batch costs less than one index pass
    match_bytes = 12 * rows + 16 * nq * ((qn + HOP - 1) // HOP)
    for sw in sweeps:
        sw["roofline_frac"] = match_bytes / (sw["batch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS
    res = {"workload": f"configs[{2 if world == 1 else 3}]: {nq} x 5 s queries vs {args.db_clips} x 30 s clips"
                        f" ({'sharded x%d, %s all_reduce MAX' % (world, 'RCCL' if args.dist_backend == 'nccl' else args.dist_backend) if world > 1 else '1 GPU'})",
            "collective": (("all_gather of the query frame values (each rank fingerprints 1/%d of the queries), "
                            "then " % world if sharded else "") + "all_reduce(MAX) of one int64 key per query")
                          if world > 1 else None,
            "coefs": 1, "tolerance": 0.001, "db_rows_local": rows, "db_clips_local": nclips_local,
            "db_build_s": t_build, "batch_queries": nq, "batch_warmup_calls": n_warm, "batch_ms": batch_ms,
            "queries_per_s": nq / (batch_ms / 1e3), "found": found,
            "latency_p50_ms": float(np.percentile(lat, 50)), "latency_p99_ms": float(np.percentile(lat, 99)),
            "latency_samples": len(lat), "latency_harness": harness,
            "latency_p50_ms_python": float(np.percentile(lat_py, 50)),
            "concurrent_callers": threads if not dist else None,
            "roofline": {"bound": "hbm", "definition": "one index pass per batch: 12 B x index rows + 16 B x query frames "
                                                       "(SURVEY 8d)", "bytes": match_bytes,
                         "achieved": match_bytes / (batch_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": match_bytes / (batch_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                         "note": "the coefs=1 vote reads only the used keys' boxes: frac > 1 = under one index pass"},
            "sweeps": sweeps}
    if world == 1 and not args.no_enrol:
        res["enrol_then_search"] = enrol_latency(args, eng, T, torch, dev, sh, p)
    if world == 1:
        res["tolerance_alternation"] = tol_alternation(args, eng, T, host_q, qn)
        res["coefs2_cache"] = coefs2_cache(args, eng, T, host_q, qn)
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = match_cpu_baseline(args, T, eng, torch, dev, sh)
        res["cpu_baseline_full_db"] = match_cpu_full_db(args, eng, torch, dev, sh, qpcm[:256].cpu().numpy())
    return res


def concurrent_searches(eng, T, clat, hq, qn, p, counts=(1, 8, 64), calls_per_count=1536):
    """Batch-1 searches per second from 1, 8 and 64 concurrent calling threads, timed from C
    (bench/tfp_latency.c: tfp_latency_threads), as the module's channel threads call
    fp_search_fingerprint_info (application_handler.c:66, :180) on one shared engine
    (fp_handler.c:1161-1169). Concurrent calls are coalesced into shared batches
    (csrc/tfp_coalesce.hpp): `batches` counts the GPU batches the calls ran as."""
    out = []
    nq = len(hq)
    for nth in counts:
        reps = max(1, calls_per_count // nth)
        sec = ctypes.c_double(0)
        found = np.zeros(nth * reps, np.int32)
        c0, b0 = ctypes.c_int64(0), ctypes.c_int64(0)
        T.lib().tfp_search_coalesce_stats(eng.handle, ctypes.byref(c0), ctypes.byref(b0))
        rc = clat.tfp_latency_threads(eng.handle, ctypes.c_void_p(hq.ctypes.data), ctypes.c_int64(qn), ctypes.c_int32(nq),
                                      ctypes.c_int32(8000), ctypes.byref(p), ctypes.c_int32(nth), ctypes.c_int32(reps),
                                      ctypes.byref(sec), ctypes.c_void_p(found.ctypes.data))
        c1, b1 = ctypes.c_int64(0), ctypes.c_int64(0)
        T.lib().tfp_search_coalesce_stats(eng.handle, ctypes.byref(c1), ctypes.byref(b1))
        if rc != 0:
            out.append({"threads": nth, "error": rc})
            continue
        out.append({"threads": nth, "calls": nth * reps, "seconds": sec.value, "searches_per_s": nth * reps / sec.value,
                    "mean_call_ms": sec.value * 1e3 * nth / (nth * reps) if nth else None,
                    "gpu_batches": b1.value - b0.value, "found": int(found.sum())})
        log(f"concurrent callers {nth}: {out[-1]['searches_per_s']:.0f} searches/s in {out[-1]['gpu_batches']} batches")
    return {"harness": "C threads over tfp_search_pcm_batch, one query each call, each query in its own tfp_host_alloc "
                       "buffer (bench/tfp_latency.c tfp_latency_threads)", "legs": out}


def enrol_latency(args, eng, T, torch, dev, sh, p, n_add=8):
    """Enrol-then-first-search at configs[2]'s 100k-clip DB: one new 30 s clip's rows added
    (tfp_index_add, as the shim's fp_craete_audio_list_info does) and a batch-1 search of a 5 s
    excerpt of it right after, timed together: the first search pays the index update. The reference's
    INSERT updates its B-tree per row (fp_handler.c:559-571, :745-753). A second engine built with
    TFP_INDEX_FULL=1 (a full re-sort per update, the round-2 behaviour) gives the figure to compare
    against.

    The new clips are full-scale white noise with uuids above every DB uuid, each above the one before
    (tests/test_gpu_configs.py: noise_clips, new_clip_uuid): their max1 values (16.19-16.25 dB) lie in
    key 16's box at tolerance 0.45 ([15.55, 16.45] dB), which holds no DB row (those are >= 16.6 dB),
    so a coefs = 1, tolerance 0.45 search of an excerpt can only be won by a new clip, and the newest
    has the greatest uuid: `new_clip_won` counts the searches that saw the clip just added. (A DB-like
    clip would not do: under the reference's trunc rule an excerpt of the synthetic audio is rarely won
    by its own clip, at any tolerance.)"""
    n_db, qn = 8000 * 30, 8000 * 5
    nf_db = (n_db + HOP - 1) // HOP
    pcm = np.random.default_rng(0x7153C3).integers(-32768, 32768, (n_add, n_db)).astype(np.int16)
    fr = eng.fingerprint_batch(pcm.reshape(-1), np.arange(n_add + 1) * n_db)
    uuids = ["ffffffff-ffff-4fff-bfff-%012x" % i for i in range(n_add)]
    pq = T.params(1, 0.45)
    for i in range(min(2, n_add)):  # untimed: this tolerance's key bitsets, built once per index version
        eng.search_pcm_batch(np.ascontiguousarray(pcm[i, :qn]), [0, qn], pq)

    def run(e, tag):
        out = []
        hits[tag] = 0
        for i, u in enumerate(uuids):
            q = np.ascontiguousarray(pcm[i, 256 * 100: 256 * 100 + qn])
            t0 = time.perf_counter()
            e.index_add(u, fr["m1"][i * nf_db:(i + 1) * nf_db], fr["m2"][i * nf_db:(i + 1) * nf_db])
            res, _ = e.search_pcm_batch(q, [0, qn], pq)
            out.append((time.perf_counter() - t0) * 1e3)
            hits[tag] += res[0] is not None and res[0]["audio_uuid"] == u
        t0 = time.perf_counter()  # the closing removals and the update they trigger (a deferred delta merges here)
        for u in uuids:
            e.index_remove(u)
        e.index_commit()
        closing[tag] = (time.perf_counter() - t0) * 1e3
        log(f"enrol-then-search ({tag}): p50 {np.percentile(out, 50):.2f} ms, new clip won {hits[tag]}/{len(uuids)}, "
            f"closing removals {closing[tag]:.2f} ms")
        return out

    hits, closing = {}, {}
    fb0, mg0 = eng.index_build_stats()
    nd0, _ = eng.index_delta_stats()
    inc = run(eng, "engine")
    fb1, mg1 = eng.index_build_stats()
    nd1, _ = eng.index_delta_stats()
    os.environ["TFP_INDEX_FULL"] = "1"
    os.environ["TFP_TEST_KNOBS"] = "1"  # (the library reads its knobs only under this switch)
    try:
        full_eng = T.Engine(eng.device)
    finally:
        del os.environ["TFP_INDEX_FULL"]
        del os.environ["TFP_TEST_KNOBS"]
    enroll(full_eng, torch, dev, sh, list(range(args.db_clips)))
    full_eng.index_commit()
    full_eng.search_pcm_batch(np.ascontiguousarray(pcm[0, :qn]), [0, qn], pq)
    full = run(full_eng, "full re-sort")
    full_eng.close()
    torch.cuda.empty_cache()
    # the same workload with a merge per update (TFP_INDEX_DELTA=0, the round-3 path): like for like
    os.environ["TFP_INDEX_DELTA"] = "0"
    os.environ["TFP_TEST_KNOBS"] = "1"
    try:
        merge_eng = T.Engine(eng.device)
    finally:
        del os.environ["TFP_INDEX_DELTA"]
        del os.environ["TFP_TEST_KNOBS"]
    enroll(merge_eng, torch, dev, sh, list(range(args.db_clips)))
    merge_eng.index_commit()
    merge_eng.search_pcm_batch(np.ascontiguousarray(pcm[0, :qn]), [0, qn], pq)
    merged = run(merge_eng, "merge per update")
    merge_eng.close()
    torch.cuda.empty_cache()
    return {"workload": f"{n_add} x (tfp_index_add of one 30 s clip + batch-1 search of a 5 s excerpt of it, coefs 1, "
                        f"tolerance 0.45) on the {args.db_clips}-clip DB, host PCM",
            "p50_ms": float(np.percentile(inc, 50)), "max_ms": float(np.max(inc)), "samples_ms": inc,
            "index_updates": {"delta_updates": nd1 - nd0, "merges": mg1 - mg0, "full_sorts": fb1 - fb0,
                              "how": "each add a delta update (the clip's rows beside the sorted index, tfp_index_delta_stats); "
                                     "the closing removals merge the delta once"},
            "closing_removals_ms": closing,
            "merge_per_update": {"p50_ms": float(np.percentile(merged, 50)), "max_ms": float(np.max(merged)),
                                 "samples_ms": merged,
                                 "how": "same workload on an engine with TFP_INDEX_DELTA=0 (each update merged into the "
                                        "sorted index at once, the round-3 path): the like-for-like comparison for the delta"},
            "new_clip_won": hits,
            "new_clips": "full-scale white noise, uuids above the DB's: only a new clip's rows lie in the query's "
                         "key box (see enrol_latency)",
            "full_resort": {"p50_ms": float(np.percentile(full, 50)), "max_ms": float(np.max(full)), "samples_ms": full,
                            "how": "same calls on an engine with TFP_INDEX_FULL=1 (every update a full radix sort of all "
                                   "staged rows + a uuid sort), the round-2 behaviour"}}


def coefs2_cache(args, eng, T, hq, qn, n_calls=100, n_add=8):
    """coefs = 2 callers (src/fp_handler.c:318-353) at the 100k-clip DB, batch-1 from host PCM:
      alternation   searches alternating tolerance 0.001 and 0.45 (the tolerance is passed per call,
                    application_handler.c:114-122): served by the clip-set cache LRU (the active
                    tolerance and three others), p50 / p99;
      after_enrol   the first search after an enrolment (tfp_index_add of one 30 s clip, then a search
                    at 0.001 or 0.45 in turn, timed together): the new clips stay in the index delta
                    and the sweep runs over the delta's own clip-set cache (its rows' clip order,
                    filtered at the search's tolerance) beside the main caches, which stay; round 6
                    first merged the delta and rebuilt the cache from the merged clip order (1.9-2.5
                    ms at 0.001, 3.2-4.4 ms at 0.45), the round-5 build sorted every box row (1.2 ms
                    at 0.001, 27 ms at 0.45, plus the merge).
    The added clips are removed again afterwards."""
    p_lo, p_hi = T.params(2, 0.001), T.params(2, 0.45)
    for i in range(4):  # untimed: both tolerances' caches at this index version
        eng.search_pcm_batch(hq[i % len(hq)], [0, qn], p_lo if i % 2 == 0 else p_hi)
    c0, w0 = eng.index_cache_stats(), eng.sweep_stats()
    lat = []
    for i in range(n_calls):
        t0 = time.perf_counter()
        eng.search_pcm_batch(hq[i % len(hq)], [0, qn], p_lo if i % 2 == 0 else p_hi)
        lat.append((time.perf_counter() - t0) * 1e3)
    c1 = eng.index_cache_stats()
    b1 = eng.index_build_stats()
    n_db = 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    pcm = np.random.default_rng(0x7153C4).integers(-32768, 32768, (n_add, n_db)).astype(np.int16)
    fr = eng.fingerprint_batch(pcm.reshape(-1), np.arange(n_add + 1) * n_db)
    uuids = ["fffffffe-ffff-4fff-bfff-%012x" % i for i in range(n_add)]
    first = []
    for i, u in enumerate(uuids):
        t0 = time.perf_counter()
        eng.index_add(u, fr["m1"][i * nf_db:(i + 1) * nf_db], fr["m2"][i * nf_db:(i + 1) * nf_db])
        eng.search_pcm_batch(hq[i % len(hq)], [0, qn], p_lo if i % 2 == 0 else p_hi)
        first.append((time.perf_counter() - t0) * 1e3)
    c2, w2 = eng.index_cache_stats(), eng.sweep_stats()
    b2 = eng.index_build_stats()
    for u in uuids:
        eng.index_remove(u)
    eng.index_commit()
    out = {"workload": f"coefs 2, batch-1 5 s host-PCM queries on the {args.db_clips}-clip DB",
           "alternation": {"calls": n_calls, "tolerances": [0.001, 0.45], "p50_ms": float(np.percentile(lat, 50)),
                           "p99_ms": float(np.percentile(lat, 99)), "max_ms": float(np.max(lat)),
                           "cache_builds": c1["builds"] - c0["builds"], "cache_hits": c1["hits"] - c0["hits"]},
           "after_enrol": {"adds": n_add, "tolerances": "0.001 / 0.45 in turn", "p50_ms": float(np.percentile(first, 50)),
                           "p99_ms": float(np.percentile(first, 99)), "max_ms": float(np.max(first)), "samples_ms": first,
                           "cache_builds_from_order": c2["from_order"] - c1["from_order"],
                           "order_merges": c2["order_merges"] - c1["order_merges"],
                           "order_full_builds": c2["order_builds"] - c1["order_builds"],
                           "index_merges": b2[1] - b1[1], "index_full_builds": b2[0] - b1[0],
                           "delta_cache_builds": c2["delta_builds"] - c1["delta_builds"],
                           "delta_sweeps": c2["delta_sweeps"] - c1["delta_sweeps"]},
           "sweep_paths": {k: w2[k] - w0[k] for k in w2},
           "harness": "python (ctypes) loop over tfp_search_pcm_batch"}
    log(f"coefs=2 cache: alternation p50 {out['alternation']['p50_ms']:.3f} p99 {out['alternation']['p99_ms']:.3f} ms; "
        f"first search after an enrolment p50 {out['after_enrol']['p50_ms']:.2f} p99 {out['after_enrol']['p99_ms']:.2f} ms")
    return out


def tol_alternation(args, eng, T, hq, qn, n_calls=200):
    """The dialplan passes the tolerance per call (application_handler.c:114-122), so two extensions
    at different tolerances alternate on the one engine: batch-1 searches (host PCM in -> result
    out) alternating tolerance 0.001 and 0.45 on the 100k-clip DB, p50 / p99. The engine keeps other
    tolerances' key ranges and bitsets beside the active ones (tfp_engine::tol_lru), and a new
    tolerance's bitsets are built without per-row atomics (launch_key_bits, round 5; the round-4
    build took 42-50 ms at 0.45). Also: the first search at a tolerance not used before (its ranges
    and bitsets built inside the call), and the first searches after the removal of an indexed clip
    (fp_handler.c:115-159: the removal merges the index; the active bitsets are carried through the
    column renumbering, the other tolerance's rebuilt). The removed clip is added back afterwards."""
    p_lo, p_hi = T.params(1, 0.001), T.params(1, 0.45)
    for i in range(4):  # untimed: both tolerances' caches
        eng.search_pcm_batch(hq[i % len(hq)], [0, qn], p_lo if i % 2 == 0 else p_hi)
    lat = []
    for i in range(n_calls):
        t0 = time.perf_counter()
        eng.search_pcm_batch(hq[i % len(hq)], [0, qn], p_lo if i % 2 == 0 else p_hi)
        lat.append((time.perf_counter() - t0) * 1e3)
    cold = []
    for tol in (0.44, 0.3):  # tolerances no search used before: ranges + bitsets built in the call
        t0 = time.perf_counter()
        eng.search_pcm_batch(hq[0], [0, qn], T.params(1, tol))
        cold.append((time.perf_counter() - t0) * 1e3)
    u = uuid_of(17)
    m1, m2 = eng.index_rows(u)
    eng.index_remove(u)
    after = []
    for i, pp in enumerate((p_hi, p_lo, p_hi, p_lo)):
        t0 = time.perf_counter()
        eng.search_pcm_batch(hq[i + 1], [0, qn], pp)
        after.append((time.perf_counter() - t0) * 1e3)
    eng.index_add(u, m1, m2)
    eng.index_commit()
    out = {"workload": f"{n_calls} batch-1 searches of 5 s host-PCM queries on the {args.db_clips}-clip DB, coefs 1, "
                       "tolerance alternating 0.001 / 0.45 per call",
           "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)), "max_ms": float(np.max(lat)),
           "first_search_at_new_tolerance_ms": {"0.44": cold[0], "0.3": cold[1]},
           "after_removal_ms": {"first (0.45: the index merge + carried bitsets)": after[0],
                                "second (0.001: its ranges and bitsets rebuilt)": after[1],
                                "third (0.45)": after[2], "fourth (0.001)": after[3]},
           "harness": "python (ctypes) loop over tfp_search_pcm_batch"}
    log(f"tolerance alternation: p50 {out['p50_ms']:.3f} ms p99 {out['p99_ms']:.3f} ms; new tolerance {cold[0]:.2f} ms; "
        f"after a removal {after[0]:.2f} / {after[1]:.2f} ms")
    return out


def match_cpu_baseline(args, T, eng, torch, dev, sh):
    """The reference's own search path on the CPU: its SQL (oracle/sql_oracle.py restates
    fp_handler.c:287-374 string for string) through SQLite 3.37, one connection, one thread, on
    a DB of --cpu-db-clips of the 30 s clips (rows as db_ctx_insert writes them: "%f" literals,
    NULL for absent keys; bulk-loaded, load not timed), queries fingerprinted by the C oracle.
    Reported: per-query latency p50/p99 (= the dialplan application's search call) and the rows
    the max1 index range scans visit per query. The GPU figures are against 100x the rows, and
    the range scans grow with the DB, so this over-states the CPU at the C3 size."""
    import oracle_py
    from sql_oracle import SqlFingerprintDB
    db_clips = args.cpu_db_clips
    n_db, qn = 8000 * 30, 8000 * 5
    nf_db = (n_db + HOP - 1) // HOP
    ids = list(range(db_clips))
    buf = torch.empty((db_clips, n_db), dtype=torch.int16, device=dev)
    eng.synth_device(SEED_DB, ids, n_db, buf.data_ptr(), stream=sh)  # same PCM as the host synth, faster
    torch.cuda.synchronize(dev)
    pcm = buf.cpu().numpy()
    del buf
    micro, _ = oracle_py.fingerprint_batch(pcm.reshape(-1), np.arange(db_clips + 1) * n_db, nthreads=16, want_db=False)
    db = SqlFingerprintDB()
    t_load = time.perf_counter()
    db.insert_rows_bulk("bench", ((uuid_of(g), micro[i * nf_db:(i + 1) * nf_db, 0], micro[i * nf_db:(i + 1) * nf_db, 1])
                                  for i, g in enumerate(ids)))
    t_load = time.perf_counter() - t_load
    m1_sorted = np.sort(micro[:, 0][micro[:, 0] != oracle_py.NULL_MICRO].astype(np.int64))
    rng = np.random.default_rng(SEED_Q + 2)
    queries, scanned = [], []
    for i in range(32):
        if i % 4 != 3:
            q = T.synth_pcm(SEED_DB, [int(rng.integers(db_clips))], qn, offsets=[256 * int(rng.integers(0, (n_db - qn) // HOP))])[0]
        else:
            q = T.synth_pcm(SEED_Q, [100000 + i], qn)[0]
        _, qdb, _ = oracle_py.fingerprint(q)
        q1 = [None if not np.isfinite(v) else float(v) for v in qdb[:, 0]]
        queries.append((q1, [None if not np.isfinite(v) else float(v) for v in qdb[:, 1]]))
        # rows of the max1 index range each frame's statement visits (coefs=1, tol 0.001)
        keys = np.trunc(np.array([0.0 if v is None else v for v in q1]))
        lo = np.array([oracle_py.fmt6(k - 0.001) for k in keys])
        hi = np.array([oracle_py.fmt6(k + 0.001) for k in keys])
        scanned.append(int((np.searchsorted(m1_sorted, hi, "right") - np.searchsorted(m1_sorted, lo, "left")).sum()))
    lat, done, found, t0 = [], 0, 0, time.perf_counter()
    while True:
        q1, q2 = queries[done % len(queries)]
        t1 = time.perf_counter()
        found += db.search(q1, q2, 1, 0.001, -1, -1) is not None
        lat.append((time.perf_counter() - t1) * 1e3)
        done += 1
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds and done >= 8:
            break
    log(f"match cpu baseline {done / dt:.1f} queries/s ({done} queries, {dt:.1f} s), p50 {np.percentile(lat, 50):.1f} ms")
    return {"value": done / dt, "unit": "queries/s", "cores": 1, "kind": "port",
            "latency_p50_ms": float(np.percentile(lat, 50)), "latency_p99_ms": float(np.percentile(lat, 99)),
            "db_clips": db_clips, "db_rows": db_clips * nf_db, "db_load_s": t_load,
            "rows_scanned_per_query_mean": float(np.mean(scanned)),
            "sample": f"{done} x 5 s queries (75 % excerpts, {found} found) vs {db_clips} x 30 s clips "
                      f"({db_clips * nf_db} rows) through the reference SQL in SQLite {__import__('sqlite3').sqlite_version}, "
                      f"1 thread, {dt:.1f} s; the GPU figures are against {args.db_clips} clips",
            "note": "the reference's SQL restated string for string (fp_handler.c:287-374), run by this image's SQLite (kind: port)"}


def match_cpu_full_db(args, eng, torch, dev, sh, qhost):
    """The same batch shape against the SAME 100,000-clip DB on the host cores: the C oracle's
    sorted-index search (oracle/oracle.c tfo_search_sorted_batch: the rows ordered by max1 as
    idx_audio_fingerprint_max1 orders them, one binary search + range scan per distinct frame
    clause, the GROUP BY / ORDER BY / LIMIT 1 of fp_handler.c:311-374) on --cpu-threads threads,
    the queries fingerprinted by the C oracle in the timed region (the GPU batch fingerprints them
    too). The rows are the device's fingerprints of the same clips (bit-exact with the oracle's,
    tests/test_gpu_configs.py), copied back untimed. Not SQLite: a B-tree-less, allocation-free
    restatement, so this is a stronger CPU than the reference's own path."""
    import oracle_py
    n_db, qn = 8000 * 30, 8000 * 5
    nf_db = (n_db + HOP - 1) // HOP
    nclips, chunk = args.db_clips, 2048
    nth = args.cpu_threads
    t0 = time.perf_counter()
    rows = np.empty((nclips * nf_db, 2), np.int32)
    buf = torch.empty((chunk, n_db), dtype=torch.int16, device=dev)
    micro = torch.empty((chunk * nf_db, 2), dtype=torch.int32, device=dev)
    for s in range(0, nclips, chunk):
        ids = list(range(s, min(nclips, s + chunk)))
        plan = eng.plan(np.arange(len(ids) + 1, dtype=np.int64) * n_db)
        eng.synth_device(SEED_DB, ids, n_db, buf.data_ptr(), stream=sh)
        eng.fingerprint_device(plan, buf.data_ptr(), micro.data_ptr(), 0, sh)
        torch.cuda.synchronize(dev)
        rows[s * nf_db:(s + len(ids)) * nf_db] = micro[:len(ids) * nf_db].cpu().numpy()
    del buf, micro
    torch.cuda.empty_cache()
    uu = np.asarray([uuid_of(g) for g in range(nclips)])
    rank = np.empty(nclips, np.int32)
    rank[np.argsort(uu)] = np.arange(nclips, dtype=np.int32)
    idx = oracle_py.SortedIndex(rows[:, 0], rows[:, 1], np.repeat(np.arange(nclips, dtype=np.int32), nf_db), rank)
    del rows
    t_build = time.perf_counter() - t0
    nq = len(qhost)
    qoff = np.arange(nq + 1, dtype=np.int64) * qn
    qfoff = np.arange(nq + 1, dtype=np.int64) * ((qn + HOP - 1) // HOP)
    done, found, t0 = 0, 0, time.perf_counter()
    while True:
        _, qdb = oracle_py.fingerprint_batch(qhost.reshape(-1), qoff, nthreads=nth)
        w, _ = idx.search_batch(qdb[:, 0], qdb[:, 1], qfoff, 1, 0.001, nthreads=nth)
        done += nq
        found += int((w >= 0).sum())
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds:
            break
    del idx
    log(f"match cpu (sorted oracle, full DB) {done / dt:.1f} queries/s on {nth} threads")
    return {"value": done / dt, "unit": "queries/s", "cores": nth, "kind": "port", "db_clips": nclips,
            "db_rows": nclips * nf_db, "setup_s": t_build,
            "sample": f"{done} x 5 s queries (the first {nq} of the GPU batch, {found} found) vs the same {nclips} x 30 s "
                      f"clips, fingerprint + search, {dt:.1f} s on {nth} threads",
            "note": "the oracle's sorted-index restatement of the reference SQL (fp_handler.c:287-374) on the full DB, "
                    "coefs=1 tol=0.001; a faster CPU path than SQLite (no B-tree, no SQL text), kind: port"}


def run_stream(args, eng, T, torch, dev, sh, rank, world, dist, barrier):
    """configs[4] (C5): live channels, 160-sample SLIN ticks, 3000 ms window (24000 samples =
    94 frames), rolling fingerprint + match against the DB. Latency = host tick in -> every
    channel's result on the host (tfp_stream_push, application_handler.c:152-185), timed from C
    (bench/tfp_latency.c, as the shim's threads call it); the same ticks through the Python
    mirror (result dicts for every channel) are reported beside it.
    N GPUs: the channels are split round-robin over the ranks and every rank holds the whole DB
    (1.13 GB at 100k clips), so a tick needs no collective; the reported per-tick
    latency is the max over ranks."""
    from tiresias_amd import Stream
    nch, W, tick, nt = args.stream_channels, 24000, 160, args.stream_ticks
    n_db = 8000 * 30
    if world > 1:  # the match leg left this rank's shard in the index: enrol the whole DB
        enroll(eng, torch, dev, sh, list(range(args.db_clips)))
        eng.index_commit()
    rng = np.random.default_rng(SEED_Q + 1)
    span = W + 2 * nt * tick  # the C-timed ticks, then the Python-timed ones
    clips = [int(rng.integers(args.db_clips)) for _ in range(nch)]
    offs = [256 * int(rng.integers(0, (n_db - span) // HOP)) for _ in range(nch)]
    mine = list(range(rank, nch, world))
    pcm = T.synth_pcm(SEED_DB, [clips[c] for c in mine], span, offsets=[offs[c] for c in mine])
    for i, c in enumerate(mine):  # every 4th channel: unrelated audio
        if c % 4 == 3:
            pcm[i] = T.synth_pcm(SEED_Q + 7, [c // 4], span)[0]
    st = Stream(eng, len(mine), W)
    p = T.params(1, 0.001)
    for t in range(W // tick):  # fill the windows (ingest only)
        st.push(pcm[:, t * tick:(t + 1) * tick])
    base = W // tick
    clat = ctypes.CDLL(os.path.join(os.path.dirname(T.LIB_PATH), "libtfp_latency.so"))
    clat.tfp_latency_stream.restype = ctypes.c_int
    pcm = np.ascontiguousarray(pcm, np.int16)
    cms = np.zeros(nt, np.float64)
    cfound = ctypes.c_int32()
    barrier()
    rc = clat.tfp_latency_stream(st._h, ctypes.c_void_p(pcm.ctypes.data), ctypes.c_int32(len(mine)), ctypes.c_int64(span),
                                 ctypes.c_int64(W), ctypes.c_int32(tick), ctypes.c_int32(nt), ctypes.byref(p),
                                 ctypes.c_void_p(cms.ctypes.data), ctypes.byref(cfound))
    assert rc == 0, rc
    found = cfound.value
    lat = cms
    plat = []
    for t in range(nt):  # the same through the Python mirror (ctypes + a result dict per channel)
        s0 = (base + nt + t) * tick
        blk = np.ascontiguousarray(pcm[:, s0:s0 + tick])
        t0 = time.perf_counter()
        st.push(blk, p)
        plat.append((time.perf_counter() - t0) * 1e3)
    plat = np.array(plat)
    if dist:
        tl = torch.tensor(lat, dtype=torch.float64, device=dev)
        dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        lat = tl.cpu().numpy()
        tl = torch.tensor(plat, dtype=torch.float64, device=dev)
        dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        plat = tl.cpu().numpy()
        tf = torch.tensor([found], dtype=torch.int64, device=dev)
        dist.all_reduce(tf)
        found = int(tf.item())
    log(f"stream: {nch} ch over {world} GPU(s), p50 {np.percentile(lat, 50):.2f} ms p99 {np.percentile(lat, 99):.2f} ms per tick")
    return {"workload": f"configs[4]: {nch} live channels, {tick}-sample ticks, {W}-sample window ({W // HOP + (W % HOP > 0)} frames), "
                        f"match vs {args.db_clips} clips every tick, "
                        + ("1 GPU" if world == 1 else f"{world} GPUs, channels split round-robin, DB replicated, no collective"),
            "ticks_timed": len(lat), "tick_latency_p50_ms": float(np.percentile(lat, 50)),
            "tick_latency_p99_ms": float(np.percentile(lat, 99)), "tick_budget_ms": 1e3 * tick / 8000,
            "tick_harness": "C loop over tfp_stream_push (bench/tfp_latency.c), the tick's samples in a tfp_host_alloc buffer",
            "tick_latency_p50_ms_python": float(np.percentile(plat, 50)),
            "fingerprints_per_tick": nch * ((W + HOP - 1) // HOP), "channels_found_last_tick": found}


def run_group(args, eng, T, torch, dev, sh, rank, world, dist):
    """The in-process device group (tfp_group_*, csrc/tfp_group.cpp) over every GPU this process
    sees (tfp_device_count): the Asterisk module is one process whose channel threads all call one
    handle (application_handler.c:180, fp_handler.c:1161-1169), and the shim (shim/fp_handler_tfp.c)
    serves them through a group. Measured through the entry points the shim calls:
      enrolment   the 100k-clip DB (configs[2]) added with tfp_group_index_add_batch (the clips'
                  rows fingerprinted on this rank's engine first), each clip on the lightest shard;
      batch       configs[3]'s 4,096 x 5 s queries from host PCM (tfp_group_search_pcm_batch: the
                  queries fingerprinted 1/N per shard, frame values exchanged peer to peer, every
                  shard searching its clips, keys max-combined), median of 5 calls;
      latency     batch-1 host-PCM searches from C (bench/tfp_latency.c), p50 / p99;
      stream      configs[4]: 512 channels through tfp_group_stream_push ticks, from C.
    Under N ranks the other ranks first release their engines (their clip shards leave the GPUs
    the group spans), meet rank 0 at a barrier, then wait on the store for as long as the leg takes.
    Rank 0 runs it; the other ranks wait on the rendezvous store (no GPU work meanwhile)."""
    store = None
    if dist:
        store = dist.distributed_c10d._get_default_store()
        if rank != 0:
            eng.close()
            torch.cuda.empty_cache()
        dist.barrier()
        if rank != 0:
            try:
                store.wait(["tfp_group_leg_done"], __import__("datetime").timedelta(hours=4))
            except Exception as ex:  # (the legs already measured stand; rank 0 prints the line)
                log(f"[rank {rank}] group leg wait ended: {ex!r}")
            return None
    try:
        return _group_leg(args, eng, T, torch, dev, sh, world)
    except Exception as ex:  # reported in the line; the fingerprint and match legs stand
        log(f"group leg failed: {ex!r}")
        return {"error": repr(ex)}
    finally:
        if store is not None:
            store.set("tfp_group_leg_done", "1")


def group_enrol_latency(g, eng, T, qn, n_add=8):
    """The shim's enrolment path at the 100k-clip DB (fp_craete_audio_list_info ->
    tfp_group_index_add, src/fp_handler.c:538-575; the clip searchable at once, :559-571): one new
    30 s clip added to the group and a batch-1 search of an excerpt of it right after
    (tfp_group_search_pcm_batch, coefs 1, tolerance 0.45), timed together, as enrol_latency times a
    bare engine. The new clip takes the middle of its uuid neighbours' tie-key gap and the shard
    gets that one key (tfp_group_tiebreak_stats: no respace, one new-clip push per add); the new
    clips are white noise whose rows alone lie in the query's key box (see enrol_latency)."""
    n_db = 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    pcm = np.random.default_rng(0x7153C5).integers(-32768, 32768, (n_add, n_db)).astype(np.int16)
    fr = eng.fingerprint_batch(pcm.reshape(-1), np.arange(n_add + 1) * n_db)
    uuids = ["fffffffd-ffff-4fff-bfff-%012x" % i for i in range(n_add)]
    pq = T.params(1, 0.45)
    g.search_pcm_batch(np.ascontiguousarray(pcm[0, :qn]), [0, qn], pq)  # untimed: this tolerance's caches
    t0s = g.tiebreak_stats()
    lat, won = [], 0
    for i, u in enumerate(uuids):
        q = np.ascontiguousarray(pcm[i, 256 * 100: 256 * 100 + qn])
        t0 = time.perf_counter()
        g.index_add(u, fr["m1"][i * nf_db:(i + 1) * nf_db], fr["m2"][i * nf_db:(i + 1) * nf_db])
        res, _ = g.search_pcm_batch(q, [0, qn], pq)
        lat.append((time.perf_counter() - t0) * 1e3)
        won += res[0] is not None and res[0]["audio_uuid"] == u
    t1s = g.tiebreak_stats()
    for u in uuids:
        g.index_remove(u)
    g.index_commit()
    out = {"workload": f"{n_add} x (tfp_group_index_add of one 30 s clip + batch-1 tfp_group_search_pcm_batch of a 5 s "
                       "excerpt of it, coefs 1, tolerance 0.45) on the group's 100k-clip DB, host PCM",
           "p50_ms": float(np.percentile(lat, 50)), "max_ms": float(np.max(lat)), "samples_ms": lat, "new_clip_won": won,
           "tie_keys": {k: t1s[k] - t0s[k] for k in t1s}, "harness": "python (ctypes) loop"}
    log(f"group enrol-then-search: p50 {out['p50_ms']:.3f} ms, won {won}/{n_add}, keys {out['tie_keys']}")
    return out


def _group_leg(args, eng, T, torch, dev, sh, world):
    from tiresias_amd import Group, GroupStream
    ndev = T.device_count()
    g = Group(list(range(ndev)))
    n_db = 8000 * 30
    nf_db = (n_db + HOP - 1) // HOP
    chunk = 2048
    t0 = time.perf_counter()
    buf = torch.empty((chunk, n_db), dtype=torch.int16, device=dev)
    micro = torch.empty((chunk * nf_db, 2), dtype=torch.int32, device=dev)
    for s0 in range(0, args.db_clips, chunk):
        ids = list(range(s0, min(args.db_clips, s0 + chunk)))
        k = len(ids)
        plan = eng.plan(np.arange(k + 1, dtype=np.int64) * n_db)
        eng.synth_device(SEED_DB, ids, n_db, buf.data_ptr(), stream=sh)
        eng.fingerprint_device(plan, buf.data_ptr(), micro.data_ptr(), 0, sh)
        torch.cuda.synchronize(dev)
        rows = micro[:k * nf_db].cpu().numpy()
        g.index_add_batch([uuid_of(i) for i in ids], np.arange(k + 1, dtype=np.int64) * nf_db, rows[:, 0], rows[:, 1])
    del buf, micro
    torch.cuda.empty_cache()
    g.index_commit()
    t_enrol = time.perf_counter() - t0
    shards = g.engine_stats()
    peers = g.peer_stats()
    log(f"group: {ndev} device(s), enrolled {args.db_clips} clips in {t_enrol:.1f} s, shards {shards}, peer access {peers}")

    nq, qn = args.queries, 8000 * 5
    hq = np.ascontiguousarray(c3_queries(eng, torch, dev, sh, nq, args.db_clips).cpu().numpy())
    off = np.arange(nq + 1, dtype=np.int64) * qn
    p = T.params(1, 0.001)
    res = None
    for _ in range(2):  # untimed: first-call allocations, caches
        res = g.search_pcm_batch(hq, off, p)[0]
    times = []
    for _ in range(5):
        t1 = time.perf_counter()
        res = g.search_pcm_batch(hq, off, p)[0]
        times.append(time.perf_counter() - t1)
    batch_ms = float(np.median(times)) * 1e3
    found = sum(r is not None for r in res)
    same = None
    if world == 1:  # this rank's engine holds the same 100k clips: the group must answer as it does
        ref = eng.search_pcm_batch(hq, off, p)[0]
        same = [None if r is None else (r["audio_uuid"], r["match_count"]) for r in ref] == \
               [None if r is None else (r["audio_uuid"], r["match_count"]) for r in res]
    log(f"group batch: {nq} queries {batch_ms:.2f} ms (host PCM in), found {found}, equal to the engine: {same}")

    clat = ctypes.CDLL(os.path.join(os.path.dirname(T.LIB_PATH), "libtfp_latency.so"))
    nl = min(args.latency_queries, nq)
    lq = np.ascontiguousarray(hq[:nl])
    for i in range(3):
        g.search_pcm_batch(lq[i], [0, qn], p)
    n_it = max(200, 10 * nl)
    out_ms = np.zeros(n_it, np.float64)
    fnd = np.zeros(n_it, np.int32)
    rc = clat.tfp_latency_group_search_pcm(g.handle, ctypes.c_void_p(lq.ctypes.data), ctypes.c_int64(qn), ctypes.c_int32(nl),
                                           ctypes.c_int32(8000), ctypes.byref(p), ctypes.c_int32(n_it),
                                           ctypes.c_void_p(out_ms.ctypes.data), ctypes.c_void_p(fnd.ctypes.data))
    assert rc == 0, rc
    out = {"workload": f"configs[3] through the shim's handle: a tfp_group over {ndev} GPU(s) in one process, "
                       f"{args.db_clips} x 30 s clips sharded by clip, {nq} x 5 s queries from host PCM",
           "n_devices": ndev, "devices": list(range(ndev)), "peer_access": peers,
           "shards_rows_clips": shards, "enrol_s": t_enrol,
           "batch_queries": nq, "batch_ms": batch_ms, "queries_per_s": nq / (batch_ms / 1e3), "found": found,
           "equal_to_engine": same,
           "latency_p50_ms": float(np.percentile(out_ms, 50)), "latency_p99_ms": float(np.percentile(out_ms, 99)),
           "latency_harness": "C loop over tfp_group_search_pcm_batch (bench/tfp_latency.c), %d calls over %d queries"
                              % (n_it, nl)}
    out["enrol_then_search"] = group_enrol_latency(g, eng, T, qn)
    assert set(GROUP_FIELDS) <= set(out), sorted(set(GROUP_FIELDS) - set(out))
    del hq
    if args.stream_channels > 0:
        nch, W, tick, nt = args.stream_channels, 24000, 160, args.stream_ticks
        rng = np.random.default_rng(SEED_Q + 1)
        span = W + nt * tick
        clips = [int(rng.integers(args.db_clips)) for _ in range(nch)]
        offs = [256 * int(rng.integers(0, (n_db - span) // HOP)) for _ in range(nch)]
        pcm = T.synth_pcm(SEED_DB, clips, span, offsets=offs)
        for c in range(3, nch, 4):
            pcm[c] = T.synth_pcm(SEED_Q + 7, [c // 4], span)[0]
        pcm = np.ascontiguousarray(pcm, np.int16)
        st = GroupStream(g, nch, W)
        for t in range(W // tick):
            st.push(pcm[:, t * tick:(t + 1) * tick])
        cms = np.zeros(nt, np.float64)
        cfound = ctypes.c_int32()
        rc = clat.tfp_latency_group_stream(st._h, ctypes.c_void_p(pcm.ctypes.data), ctypes.c_int32(nch), ctypes.c_int64(span),
                                           ctypes.c_int64(W), ctypes.c_int32(tick), ctypes.c_int32(nt), ctypes.byref(p),
                                           ctypes.c_void_p(cms.ctypes.data), ctypes.byref(cfound))
        assert rc == 0, rc
        st.close()
        out["stream"] = {"workload": f"configs[4]: {nch} channels, {tick}-sample ticks, {W}-sample window, channels split "
                                     f"over the group's {ndev} shard(s) (channel c on shard c mod N), window frame values "
                                     f"copied to the other shards, every shard matching its clips",
                         "ticks_timed": nt, "tick_latency_p50_ms": float(np.percentile(cms, 50)),
                         "tick_latency_p99_ms": float(np.percentile(cms, 99)), "channels_found_last_tick": cfound.value,
                         "tick_harness": "C loop over tfp_group_stream_push (bench/tfp_latency.c)"}
        log(f"group stream: p50 {out['stream']['tick_latency_p50_ms']:.2f} ms")
    g.close()
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
