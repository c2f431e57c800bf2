#!/usr/bin/env python3
"""Flagship benchmark: ALS batch-layer ratings/sec on MI355X (BASELINE.json).

``python bench.py --gpus N --steps K --warmup W``; for N > 1 launch one rank per GPU with
``torch.distributed.run`` (RCCL over xGMI).  A *step* is one full ALS iteration of the batch
layer's trainer -- item half-step + user half-step: all-reduce of the partial Gramians,
the fused HIP gather/MFMA-Gramian/Cholesky solve of every owned row, and the all-gather of
the new bf16 factor shard -- over the whole synthetic ratings matrix.

Config (BASELINE.json "ALS rank=64 bf16 on 25M synthetic ratings, 1 MI355X"): implicit ALS,
rank 64, lambda 0.001, alpha 1 (reference defaults except rank), bf16 factors with fp32
accumulation and fp32 solves.  Weak scaling: every rank owns 25M ratings of its own 162,541
users (MovieLens-25M-like shape) over a shared catalogue of 59,047 items with skewed
popularity; the all-to-all that repartitions ratings by item happens once, before timing.

Prints ONE JSON line (rank 0).  ``value`` = total ratings processed per second over all
ranks = (global nnz * K) / max-over-ranks(time of K steps).  Extra fields report the
speed-layer fold-in latency for a 10k-event micro-batch (the second half of the metric).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _gen_ratings(n_local_users: int, n_items: int, nnz: int, rank: int, seed: int, device):
    """Unique (user, item, strength) triples for this rank's users, skewed activity/popularity."""
    g = torch.Generator(device=device)
    g.manual_seed(seed * 7919 + rank)
    u_lo = rank * n_local_users
    have = torch.empty(0, dtype=torch.int64, device=device)
    want = nnz
    while have.numel() < want:
        m = int((want - have.numel()) * 1.25) + 1024
        u = (n_local_users * torch.rand(m, generator=g, device=device).pow(1.3)).to(torch.int64)
        i = (n_items * torch.rand(m, generator=g, device=device).pow(2.5)).to(torch.int64)
        u = u.clamp_(0, n_local_users - 1)
        i = i.clamp_(0, n_items - 1)
        have = torch.unique(torch.cat([have, u * n_items + i]))
    keep = torch.randperm(have.numel(), generator=g, device=device)[:want]
    key = have[keep]
    users = torch.div(key, n_items, rounding_mode="floor") + u_lo
    items = key % n_items
    strength = torch.randint(1, 11, (want,), generator=g, device=device).to(torch.float32) * 0.5
    return users, items, strength


# BASELINE.json configs this bench covers (weak scaling: per-GPU shares of the named totals)
PRESETS = {
    # "ALS rank=64 bf16 on 25M synthetic ratings, 1 MI355X"
    "c2": dict(rank_k=64, ratings_per_gpu=25_000_000, users_per_gpu=162_541, items=59_047,
               precision="bf16"),
    # "ALS rank=128 on 1B synthetic ratings, 8xMI355X": 125M ratings of 1.25M users per GPU
    # over a shared 500k-item catalogue (1B ratings / 10M users at 8 GPUs)
    # (no dtype named: MLlib's fp32 factors, carried as bf16 hi|lo pairs)
    "c3": dict(rank_k=128, ratings_per_gpu=125_000_000, users_per_gpu=1_250_000,
               items=500_000, precision="fp32"),
}


# effective one-direction bandwidth of one xGMI link (7 links x ~153 GB/s per GPU, both
# directions): what one peer-to-peer stream of stores sustains, an assumption of the estimate
XGMI_LINK_GBPS = 64.0


def exchange_schedule(trainer, halfstep_ms: dict, W: int, elem: int) -> dict:
    """Exposed factor-exchange time per iteration estimated from the per-link schedule of the
    range-by-range exchange (range c moves while range c + 1 is solved; the last range's
    transfer is exposed, and so is any range whose transfer outlasts the next solve):

    * peer push (parallel/ipc.py IpcAllGather): a range goes to the W - 1 peers over W - 1
      different links at once, so it takes range_bytes / link bandwidth;
    * ring all-gather: every byte of the W - 1 other ranks' ranges crosses this rank's one
      inbound ring link, (W - 1) range_bytes / link bandwidth."""
    bw = XGMI_LINK_GBPS * 1e9
    out = {"link_gbps_assumed": XGMI_LINK_GBPS}
    for half, lay in (("items", trainer.lay_i), ("users", trainer.lay_u)):
        rb = lay.cr * trainer.kp * elem
        solve_c = halfstep_ms.get("%s_solve_ms" % half, 0.0) / max(1, lay.C)
        for how, t in (("push", rb / bw * 1e3), ("ring", (W - 1) * rb / bw * 1e3)):
            exposed = t + sum(max(0.0, t - solve_c) for _ in range(lay.C - 1))
            out["%s_%s_ms" % (half, how)] = exposed
        out["%s_range_bytes" % half] = rb
        out["%s_ranges" % half] = lay.C
        out["%s_solve_per_range_ms" % half] = solve_c
    out["push_ms_per_iteration"] = out["items_push_ms"] + out["users_push_ms"]
    out["ring_ms_per_iteration"] = out["items_ring_ms"] + out["users_ring_ms"]
    return out


def emulate(args) -> int:
    """--emulate-world W --emulate-rank r: rank r's per-rank workload of a W-GPU weak-scaling
    run on one GPU (see the argument's help).  Prints one JSON line (not the headline
    metric: the collectives are not executed, their payloads are reported)."""
    from oryx_amd.parallel import dist
    from oryx_amd.models.als.trainer import ALSTrainer
    W, R = int(args.emulate_world), int(args.emulate_rank)
    if not 0 <= R < W:
        raise SystemExit("--emulate-rank must be in [0, --emulate-world)")
    dev = dist._pick_device(0, args.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    ctx = dist.DistContext(rank=R, world_size=W, device=dev, emulated=True)
    t0 = time.perf_counter()
    bu, bi = [[], [], []], [[], [], []]
    nnz_world = 0
    for q in range(W):
        u, i, s = _gen_ratings(args.users_per_gpu, args.items, args.ratings_per_gpu, q,
                               args.seed, dev)
        nnz_world += int(u.numel())
        mu, mi = (u % W) == R, (i % W) == R
        for dst, m in ((bu, mu), (bi, mi)):
            dst[0].append(u[m])
            dst[1].append(i[m])
            dst[2].append(s[m])
        del u, i, s
    by_user = [torch.cat(c) for c in bu]
    by_item = [torch.cat(c) for c in bi]
    gen_s = time.perf_counter() - t0
    trainer = ALSTrainer(args.rank_k, lam=0.001, alpha=1.0, implicit=bool(args.implicit),
                         ctx=ctx, seed=args.seed, precision=args.precision,
                         gather_chunks=args.gather_chunks)
    trainer.prepare_routed(by_user, by_item, args.users_per_gpu * W, args.items)
    nnz_u, nnz_i = int(by_user[0].numel()), int(by_item[0].numel())
    del by_user, by_item
    trainer.init_factors()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        trainer.iterate(1)
    sync()
    t0 = time.perf_counter()
    trainer.iterate(args.steps)
    sync()
    ms = (time.perf_counter() - t0) * 1e3 / max(1, args.steps)
    halfstep_ms = trainer.phase_breakdown(3)
    elem = 4 if trainer.split else 2
    kp = trainer.kp
    # what one iteration's collectives would move on this rank (ring algorithms: an
    # all-gather sends this rank's shard and receives W - 1 others; an all-reduce of B bytes
    # sends and receives 2 (W - 1) / W B)
    gram = kp * kp * 4
    ag = {"items": trainer.lay_i.local_rows * kp * elem,
          "users": trainer.lay_u.local_rows * kp * elem}
    coll = {"allreduce_gramian_bytes": 2 * gram,
            "allgather_send_bytes": ag["items"] + ag["users"],
            "allgather_recv_bytes": (W - 1) * (ag["items"] + ag["users"]),
            "allreduce_wire_bytes": int(2 * 2 * (W - 1) / W * gram)}
    # xGMI: 7 links x ~153 GB/s per GPU; a ring all-gather is bound by one link per peer
    # step, so the received bytes over ~64 GB/s of effective ring bandwidth (RCCL's
    # multi-channel rings reach roughly that per GPU pair) bounds the exposed exchange
    coll["allgather_ring_est_ms"] = coll["allgather_recv_bytes"] / 64e9 * 1e3
    coll["exposed_exchange_est"] = exchange_schedule(trainer, halfstep_ms, W, elem)
    rec = {
        "metric": "ALS per-rank iteration time, emulated %d-GPU weak scaling (rank %d)" % (W, R),
        "emulated": True, "world": W, "rank": R, "preset": args.preset,
        "ms_per_step": ms, "steps": args.steps, "warmup": args.warmup,
        "halfstep_ms": halfstep_ms,
        "ratings_world": nnz_world, "ratings_user_csr": nnz_u, "ratings_item_csr": nnz_i,
        "rows": {"users": trainer.u_hi - trainer.u_lo, "items": trainer.i_hi - trainer.i_lo,
                 "gather_chunks_items": trainer.lay_i.C, "gather_chunks_users": trainer.lay_u.C},
        "collectives_per_iteration": coll,
        "per_gpu_ratings_per_s": nnz_world / W * 1e3 / ms,
        "config": {"rank_k": args.rank_k, "precision": args.precision,
                   "ratings_per_gpu": args.ratings_per_gpu, "users_per_gpu": args.users_per_gpu,
                   "items": args.items},
        "generate_s": gen_s, "prepare_s": trainer.timings.get("prepare_s"),
        "solve_failures": trainer.failures,
        "peak_hbm_gib": (torch.cuda.max_memory_allocated(dev) / 2 ** 30
                         if dev.type == "cuda" else None),
    }
    print(json.dumps(rec), flush=True)
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--preset", choices=sorted(PRESETS), default="c2")
    ap.add_argument("--rank-k", type=int, default=None, help="ALS rank (features)")
    ap.add_argument("--ratings-per-gpu", type=int, default=None)
    ap.add_argument("--users-per-gpu", type=int, default=None)
    ap.add_argument("--items", type=int, default=None)
    ap.add_argument("--precision", choices=["bf16", "fp32"], default=None,
                    help="factor operand precision (fp32 = bf16 hi|lo split operands)")
    ap.add_argument("--implicit", type=int, default=1)
    ap.add_argument("--speed-events", type=int, default=10_000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--gather-chunks", type=int, default=None,
                    help="row ranges per half-step factor exchange (default: trainer's)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one GPU plays rank --emulate-rank of a W-rank weak-scaling run: it "
                         "builds that rank's exact post-all-to-all CSRs (from every rank's "
                         "generated ratings) and full-size gathered factor buffers, runs the "
                         "half-steps with collectives that move nothing, and reports their "
                         "times plus the bytes each collective would move")
    ap.add_argument("--emulate-rank", type=int, default=0)
    args = ap.parse_args(argv)
    for key, val in PRESETS[args.preset].items():
        if getattr(args, key) is None:
            setattr(args, key, val)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if args.emulate_world > 1:
        return emulate(args)
    from oryx_amd.parallel import launch
    rc = launch.relaunch_if_needed(os.path.abspath(__file__), argv, args.gpus)
    if rc is not None:
        return rc
    from oryx_amd.parallel import dist
    from oryx_amd.models.als.trainer import ALSTrainer
    from oryx_amd.ops import als as als_ops
    from oryx_amd.utils import mathx

    ctx = dist.init_from_env(device=args.device)
    dev = ctx.device
    W = ctx.world_size
    n_users = args.users_per_gpu * W
    users, items, strength = _gen_ratings(args.users_per_gpu, args.items, args.ratings_per_gpu,
                                          ctx.rank, args.seed, dev)
    trainer = ALSTrainer(args.rank_k, lam=0.001, alpha=1.0, implicit=bool(args.implicit),
                         ctx=ctx, seed=args.seed, precision=args.precision,
                         gather_chunks=args.gather_chunks)
    trainer.prepare(users, items, strength, n_users, args.items)
    del users, items, strength
    trainer.init_factors()
    nnz_local = torch.tensor([float(trainer.local_nnz)], dtype=torch.float64, device=dev)
    dist.all_reduce_sum(nnz_local, ctx)
    global_nnz = int(nnz_local.item())

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        trainer.iterate(1)
    sync()
    dist.barrier(ctx)
    sync()
    if os.environ.get("ORYX_BENCH_TIMED_MARK"):
        # (scripts/speed_under_load.py: another process waits for the timed loop to start)
        open(os.environ["ORYX_BENCH_TIMED_MARK"], "w").close()
    t0 = time.perf_counter()
    trainer.iterate(args.steps)
    sync()
    dist.barrier(ctx)
    sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if ctx.is_distributed:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / max(1, args.steps)
    ratings_per_sec = global_nnz * args.steps / elapsed

    # per-half-step phases (Gramian + YtY all-reduce / solve / exposed factor exchange) from
    # CUDA events over 3 extra iterations -- untimed, for diagnosing scaling runs
    halfstep_ms = trainer.phase_breakdown(3)

    # ---- speed layer: one micro-batch of new events through the real speed-layer update
    # (ALSSpeedModelManager.build_updates: native parse, aggregation, Gramian inverses, the
    # fused HIP fold-in, native UP-message formatting) against the trained model, and the
    # append of its UP block to an update log (the speed layer's producer.send_block):
    # median and p90 over 12 repetitions after 2 warm-ups (rank 0's GPU)
    speed_ms = speed_p90 = foldin_ms = speed_phases = n_updates = None
    # full factors on every rank (a collective), used by rank 0's speed-layer model
    f = trainer.factors() if args.speed_events > 0 else None
    if ctx.is_main and args.speed_events > 0:
        import numpy as np
        from oryx_amd.api import Dataset
        from oryx_amd.models.als.speed import ALSSpeedModel, ALSSpeedModelManager
        from oryx_amd.utils import config as cfg
        k = args.rank_k
        Xh, Yh = f.X.cpu().numpy(), f.Y.cpu().numpy()
        mgr = ALSSpeedModelManager(cfg.get_default())
        model = ALSSpeedModel(k, bool(args.implicit), dev)
        model.X.set_vectors(["U%d" % j for j in range(len(Xh))], Xh)
        model.Y.set_vectors(["I%d" % j for j in range(len(Yh))], Yh)
        mgr.model = model
        g = np.random.default_rng(99)
        B = args.speed_events
        now = int(time.time() * 1000)
        lines = ["U%d,I%d,%.2f,%d" % (a, b, v, now) for a, b, v in
                 zip(g.integers(0, len(Xh), B).tolist(), g.integers(0, len(Yh), B).tolist(),
                     (g.random(B) * 4 + 0.5).tolist())]
        # the micro-batch as the speed layer drains it from the input log: one TextLines
        # buffer (layers/common.drain_dataset), not Python strings
        from oryx_amd.textlines import TextLines
        ds = Dataset.from_values(TextLines.from_strings(lines))
        import shutil
        import tempfile
        from oryx_amd.layers.speed import publish_blocks
        from oryx_amd.transport.producer import LogTopicProducer
        logdir = tempfile.mkdtemp(prefix="oryx_bench_speed_")
        producer = LogTopicProducer("log:" + logdir, "OryxUpdate", async_=False,
                                    max_message=1 << 30)
        times, phases = [], []
        try:
            for rep in range(14):
                # a new micro-batch always follows a change of the factors (the previous
                # batch's own UP rows): the Gramian inverses are recomputed every time
                model.X.version += 1
                # micro-batches arrive one per speed interval (oryx.speed.streaming.
                # generation-interval-sec, seconds): 50 ms of idle time between reps (untimed)
                # lets the update log's tail preallocation run as it does between intervals
                time.sleep(0.05)
                sync()
                t1 = time.perf_counter()
                # the speed layer's path: blocks of UP rows assembled while the previous
                # block is appended to the update log (layers/speed.py publish_blocks)
                pub: dict = {}
                n_updates = publish_blocks(producer, mgr.build_update_blocks(ds), pub)
                t3 = time.perf_counter()
                if rep >= 2:
                    times.append((t3 - t1) * 1e3)
                    ph = dict(mgr.last_phase_ms)
                    ph["publish_write"] = pub.get("write_ms", 0.0)
                    ph["publish_tail"] = pub.get("tail_ms", 0.0)
                    phases.append(ph)
        finally:
            producer.close()
            shutil.rmtree(logdir, ignore_errors=True)
        speed_ms = float(np.median(times))
        speed_p90 = float(np.percentile(times, 90))
        speed_phases = {k: float(np.median([p_.get(k, 0.0) for p_ in phases]))
                        for k in phases[0]}
        foldin_ms = speed_phases.get("foldin")

    info = dist.run_info(ctx)
    peak = torch.tensor([float(torch.cuda.max_memory_allocated(dev)) if dev.type == "cuda"
                         else 0.0], dtype=torch.float64, device=dev)
    if ctx.is_distributed:
        torch.distributed.all_reduce(peak, op=torch.distributed.ReduceOp.MAX)
    if ctx.is_main:
        rec = {
            "metric": "ALS batch-layer ratings/sec + speed-layer model-update latency, 1/2/4/8 MI355X",
            "value": ratings_per_sec,
            "unit": "ratings/s",
            "n_gpus": W,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (power-law users x items, unique pairs, strengths 0.5..5), "
                    "random-init unit-Gaussian factors",
            "config": {
                "model": "ALS implicit rank=%d lambda=0.001 alpha=1 (MLlib normal equations)"
                         % args.rank_k,
                "global_batch": global_nnz,
                "seq_len": None,
                "parallelism": "dp%d (user/item row shards, RCCL all-reduce YtY + all-gather "
                               "factors)" % W,
                "ratings_per_gpu": args.ratings_per_gpu,
                "users": n_users,
                "items": args.items,
                "step": "1 ALS iteration (items+users half-steps)",
                "preset": args.preset,
            },
            "world_size": info["world_size"],
            "backend": info["backend"],
            "ipc_allreduce": info.get("ipc_allreduce", False),
            "allgather": info.get("allgather"),
            "allgather_selftest": info.get("allgather_selftest"),
            "rank_devices": [r.get("current_device", r["device"]) for r in info["ranks"]],
            "peak_hbm_gib_per_rank": float(peak.item()) / 2**30,
            "halfstep_ms": halfstep_ms,
            "speed_layer_update_ms": speed_ms,
            "speed_layer_update_p90_ms": speed_p90,
            "speed_layer_reps": 12,
            "speed_layer_events": args.speed_events,
            "speed_layer_update_messages": n_updates,
            "speed_layer_foldin_ms": foldin_ms,
            "speed_layer_phase_ms": speed_phases,
            "speed_layer_path": "ALSSpeedModelManager.build_update_blocks (parse, aggregate, "
                                "inverses, fused HIP fold-in, UP "
                                "formatting, assembly) + the UP block's append to the update "
                                "log (layers/speed.py publish_blocks); end to end, median of "
                                "12",
            "solve_failures": trainer.failures,
            "gather_chunks": {"items": trainer.lay_i.C, "users": trainer.lay_u.C},
        }
        print(json.dumps(rec), flush=True)
    if ctx.is_distributed:
        dist.barrier(ctx)
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
