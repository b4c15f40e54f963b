#!/usr/bin/env python3
"""bench.py — fused product+sum-out throughput (factor-entries/s) on MI355X.

Workload (BASELINE config 5 restated): one VE bucket of a
4-state Potts model,  msg(S_1..S_w, y) = sum_x m(x, S_1..S_w) * f(x, y),  all
cards k = 4, w = 14, fp32  =>  4^16 = 4.29e9 factor-entries per step, inputs
resident in HBM.  With --gpus N every rank evaluates its own independent bucket
of that shape (its own seed): weak scaling, fixed work per GPU, no data-path
collective, one barrier + max-reduce of the timer.  Checks: the checksum of
checksums (sum of the output = sum_x rowsum(m)_x * rowsum(f)_x) and an exact
spot check of 512 random output entries against the same arithmetic in torch
(fp32 products, sums in the reference's order).

A "step" = one fused bucket (one kernel launch) through the C ABI
(bnpp_bucket_eliminate) on torch's current stream.  Roofline: algorithmic bytes
= 4 B x (|m| + |f| + |out|) per launch over the kernel's average duration (HIP
events, same stream) against 8.0 TB/s.  CPU baseline: the reference's own
Factor::product + Factor::sum_out (oracle/_ref/ref_harness micro, compiled from
the reference sources), or the oracle restatement if that binary is absent,
single core, on a bounded sample of the same bucket shape.

"mar": the metric's second half on its own instance -- all marginals of the
32x32 Ising grid UAI (BASELINE config 3) through the checkpointed two-pass
bucket tree (column-sweep order, width 32, fp32), split over the ranks by
chain segments; wall-clock like the reference's uptime, warm (the identical
second call on the context: the cached job relaunched -- no ordering or
planning -- in its arena; "cold_wall_ms" = the first call, which orders,
plans, allocates the arena and loads the kernels), each with its phase split
(bnpp_last_timing).  It runs after the bucket and the CPU
baseline: HBM freed by an earlier process is cleared by the driver in the
background for several seconds, and a first touch before that waits for it
(profiles/r03_cold_after_free.jsonl).  "check": P(x_t = 0) of three targets
against Z(x_t = 0) / Z from conditioned partitions on the same context (rank
0, after the timed calls).  The reference cannot run this instance (min-fill
width 46), so its time is bounded from below by n_vars x the column-sweep
PR's factor-entries at the measured cpu_baseline rate.  "secondary": 10x10
(reference-runnable): the reference's own BN::marginals (oracle/_ref
ref_harness mar, one core, taskset) timed in this run, beside the GPU
per-target and bucket-tree MAR (first call on a fresh model, as the
reference's one-shot uptime; relaunch beside it), with the largest difference
between them.  "fp64_bucket": the same k=4, w=14 bucket in the reference's
precision (bit-exact path; 17.2 GB per launch), with its own roofline
fraction.  "mar_f64": the 32x32 MAR in the reference's precision (fp64 split
runs, 32-GiB messages), cold and warm, checked at 1e-11.

N GPUs: `python bench.py --gpus N` outside a launcher starts the N ranks
itself (python -m torch.distributed.run as a child process, before any GPU
call); under a launcher every rank checks WORLD_SIZE == --gpus.  The record
names "world_size" and "backend".  From 4 ranks the message-sliced tree MAR
(DESIGN §6), the scaling MAR of the north star, runs too, timed the same way
(max over ranks, cold and warm); the faster of the two schemes is the
record's "mar" and the other stands beside it ("mar_segment", or
mar["sliced"]).  cpu_baseline runs on rank 0 at every world size.
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "bn-pp_amd", "python"))

METRIC = "factor-entries/sec on fused product+sum-out; MAR wall-clock on 32x32 grid UAI"
HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md chip table (spec)


def host_cpu():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def cpu_baseline(k: int, w_cpu: int, reps: int):
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    sample = "m(x,S_1..S_%d)*f(x,y)->sum_x, k=%d, fp64, %d rep(s): %d factor-entries" % (
        w_cpu, k, reps, k ** (w_cpu + 2) * reps)
    if os.path.exists(harness):
        out = subprocess.run(["taskset", "-c", "0", harness, "micro", str(k), str(w_cpu), str(reps)],
                             capture_output=True, text=True, check=True, timeout=600).stdout
        kv = dict(line.split() for line in out.splitlines() if len(line.split()) == 2)
        rec = {"value": float(kv["entries_per_s"]), "unit": "factor-entries/s", "cores": 1, "kind": "reference",
               "sample": sample + " (reference Factor::product + sum_out, compiled from /root/reference/code; "
                                  "taskset -c 0)", "seconds": float(kv["seconds"])}
    else:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import refcpu
        eps, sec = refcpu.micro_bucket(k, w_cpu, reps)
        rec = {"value": eps, "unit": "factor-entries/s", "cores": 1, "kind": "port",
               "sample": sample + " (oracle restatement)", "seconds": sec}
    rec.update(host_cpu())
    return rec


def reference_mar(name: str):
    """The reference's own BN::marginals on a bundled instance (per-target VE,
    model.cpp:326-334, min-fill), one core: (uptime ms, {var: [p..]}) or None."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    path = os.path.join(REPO, "tests", "golden", "models", name)
    out = subprocess.run(["taskset", "-c", "0", harness, "mar", path, "-", "mf"], capture_output=True, text=True,
                         check=True, timeout=600).stdout
    marg, up = {}, None
    for line in out.splitlines():
        if line.startswith("M") and "|" in line:
            head, _, vals = line.split("|")
            marg[int(head.split()[0][1:])] = [float(x) for x in vals.split()]
        elif line.startswith("uptime_ms"):
            up = float(line.split()[1])
    return up, marg


def mar_wallclock(ctx, rank, world, dist, dev, rows, cols, dtype_name, column_order):
    """Second half of the metric: MAR wall-clock.  All marginals of an R x C
    Ising grid (BN::marginals, model.cpp:303-346) by the two-pass bucket tree
    (bnpp_marginals_tree_part): on one GPU the whole tree; on N GPUs part r of
    N (a contiguous segment of the chain: its forward prefix, the backward
    messages down to it, checkpointed recomputation inside it), assembled by one
    all-reduce.  Timed like the reference's uptime (ordering + planning + device
    run + normalise), max over ranks."""
    import torch
    import bnpp
    from bnpp import synth, dist as bdist

    dt = bnpp.F32 if dtype_name == "f32" else bnpp.F64
    m = bnpp.Model.from_dict(synth.ising_grid(rows, cols, seed=0))
    order = [r * cols + c for c in range(cols) for r in range(rows)] if column_order else None
    def timed():
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        mg = bdist.sharded_tree_marginals(ctx, m, rank, world, dist, {}, "mf", dt, order)
        ms = (time.perf_counter() - t0) * 1e3
        if dist is not None:
            tt = torch.tensor([ms], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ms = tt.item()
        return mg, ms

    # first: the first call of this dtype on the context (orders, plans, loads
    # kernels; allocates the arena unless a cached one of another call is big
    # enough); warm: the same call again, the cached job relaunched in its arena
    # (a serving process keeps it)
    marg, first_ms = timed()
    first_phases = bnpp.last_timing()
    marg2, ms = timed()
    warm_phases = bnpp.last_timing()
    assert marg2 == marg
    name = "ising%dx%d" % (rows, cols)
    rec = {"instance": "%s all marginals, bucket tree, %s order, %s" % (
               name, "column-sweep (width %d)" % rows if column_order else "min-fill", dtype_name),
           "wall_ms": ms, "n_gpus": world, "p_var0": marg[0],
           "max_sum_err": max(abs(sum(p) - 1.0) for p in marg.values())}
    if first_phases.get("arena_reused"):
        # the first call ran in an arena an earlier call left cached: not a
        # one-shot figure.  The one-shot (cold) call is made after freeing
        # every cached arena: it allocates its own and waits, in that
        # hipMalloc, for the driver to clear the HBM just freed
        ctx.trim()
        marg3, cold_ms = timed()
        cold_phases = bnpp.last_timing()
        assert marg3 == marg
        rec["warm_arena_first_call_ms"] = first_ms
        rec["cold_note"] = ("cold = fresh context state: every cached arena freed (ctx.trim) right before, so the "
                            "arena hipMalloc waits for the driver to clear that HBM; warm_arena_first_call_ms = "
                            "the first call of this dtype, run in the arena the fp32 MAR left cached")
        phases = {"warm_arena_first_call": first_phases, "cold": cold_phases, "warm": warm_phases}
    else:
        cold_ms, cold_phases = first_ms, first_phases
        rec["cold_note"] = ("cold = the first MAR call in the process: orders, plans, allocates its arena (waiting "
                            "there for the driver to clear HBM freed shortly before by any process), loads kernels")
        phases = {"cold": cold_phases, "warm": warm_phases}
    rec.update({"cold_wall_ms": cold_ms, "cold_over_warm": cold_ms / ms,
                # the cold call's arena hipMalloc, where it waits for the driver to
                # clear HBM freed before it (by any process; DESIGN §7 "Cold calls")
                "cold_arena_alloc_ms": cold_phases.get("arena_alloc_ms"),
                "cold_wall_ms_excl_arena_alloc": cold_ms - (cold_phases.get("arena_alloc_ms") or 0.0),
                "phases_ms": phases})
    if rank == 0:
        # P(x_t = 0) = Z(x_t = 0) / Z, each Z by one conditioned VE (BN::partition)
        lz = bnpp.partition(ctx, m, {}, "mf", dt, order=order)[0]
        tol = 1e-6 if dt == bnpp.F32 else 1e-11
        errs = {}
        for t in (0, (rows // 2) * cols + cols // 2, rows * cols - 1):
            lz0 = bnpp.partition(ctx, m, {t: 0}, "mf", dt, order=order)[0]
            errs[str(t)] = abs(10 ** (lz0 - lz) - marg[t][0])
        rec["check"] = {"method": "P(x_t=0) vs Z(x_t=0)/Z from conditioned partitions", "abs_err": errs,
                        "max_abs_err": max(errs.values()), "tolerance": tol,
                        "ok": max(errs.values()) <= tol}
    rec["_model"] = (m, order, dt, marg)                   # for the sliced leg
    # the reference cannot run it (min-fill width 46 at 32x32); lower bound
    # (filled in by reference_bound once the CPU rate is measured): one VE
    # per variable, each at least the column-sweep PR's factor-entries
    rec["_bound"] = (m.n_vars, bnpp.plan_stats(m, 0, {}, "mf", dtype=dt, order=order)[0], rows)
    return rec


def sliced_mar(ctx, rank, world, dist, dev, m, order, dt, marg_ref):
    """The same marginals with every message sliced over the ranks
    (bnpp.dist.sliced_tree_marginals): wall-clock max over ranks,
    cold and warm, and the largest difference from the segment scheme's
    marginals.  Guarded: its collectives run in process groups with a 120-s
    timeout, and any failure is recorded instead of ending the bench."""
    import torch
    from bnpp import dist as bdist

    def timed():
        dist.barrier()
        t0 = time.perf_counter()
        mg, st = bdist.sliced_tree_marginals(ctx, m, rank, world, dist, {}, "mf", dt, order, timeout_s=120)
        ms = (time.perf_counter() - t0) * 1e3
        tt = torch.tensor([ms], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return mg, st, tt.item()

    try:
        _, _, cold = timed()
        mg, st, warm = timed()
        diff = max(max(abs(a - b) for a, b in zip(mg[t], marg_ref[t])) for t in marg_ref)
        return {"wall_ms": warm, "cold_wall_ms": cold, "exchanges_per_call": st["calls"],
                "bytes_sent_per_rank": st["bytes_sent"], "max_abs_diff_vs_segment_scheme": diff,
                "ok": diff <= (2e-6 if dt == 1 else 1e-11)}
    except Exception as e:                                  # recorded, not fatal
        return {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}


def secondary_mar(ctx, name: str, with_reference: bool):
    """A reference-runnable MAR (min-fill, fp64): the GPU per-target VE (the
    reference's algorithm, bit-exact path) and the GPU bucket tree, and --
    rank 0 at N=1 -- the reference's own BN::marginals timed in this run on
    one core.  Like for like: the reference's uptime is a one-shot process
    (ordering + VE + normalise, model.cpp:303-346), so the speed-ups divide it
    by each GPU path's FIRST call on a freshly loaded model (ordering,
    planning, source upload, run, fetch); the relaunch of the same call (the
    context's cached job: no ordering or planning) is reported beside it."""
    import bnpp
    path = os.path.join(REPO, "tests", "golden", "models", name)
    rec = {"instance": "%s all marginals, min-fill, f64" % name}
    res = {}
    for kind, fn in (("per_target", lambda m: bnpp.marginals(ctx, m, {}, "mf", bnpp.F64)),
                     ("bucket_tree", lambda m: bnpp.marginals_tree(ctx, m, {}, "mf", bnpp.F64))):
        m = bnpp.Model.load(path)                      # a new model: nothing cached for it
        t0 = time.perf_counter()
        res[kind], _ = fn(m)
        rec[kind + "_wall_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        fn(m)
        rec[kind + "_relaunch_wall_ms"] = (time.perf_counter() - t0) * 1e3
    rec["max_abs_diff_tree_vs_per_target"] = max(abs(a - b) for t in res["per_target"]
                                                 for a, b in zip(res["per_target"][t], res["bucket_tree"][t]))
    if with_reference:
        r = reference_mar(name)
        if r is not None:
            up, rm = r
            rec.update({"reference_cpu_ms": up, "reference_kind": "reference (oracle/_ref ref_harness mar, "
                                                                  "compiled from /root/reference/code, taskset -c 0)",
                        "speedup_per_target": up / rec["per_target_wall_ms"],
                        "speedup_bucket_tree": up / rec["bucket_tree_wall_ms"],
                        "speedup_note": "reference one-shot uptime / GPU first-call wall-clock",
                        "max_abs_diff_vs_reference": max(abs(a - b) for t in rm
                                                         for a, b in zip(rm[t], res["per_target"][t]))})
    # fp64 both ways: the per-target path is the reference's arithmetic, the
    # tree associates the sums differently
    rec["tolerance"] = 1e-12
    rec["ok"] = (rec["max_abs_diff_tree_vs_per_target"] <= 1e-12 and
                 rec.get("max_abs_diff_vs_reference", 0.0) <= 1e-12)
    return rec


def reference_bound(rec, cpu_rate):
    """Reference MAR lower bound at the reference's measured product+sum-out
    rate on this host (see mar_wallclock)."""
    n_vars, pr, rows = rec.pop("_bound")
    if not cpu_rate:                                       # no CPU baseline measured in this run: no bound
        return
    lb = n_vars * pr / cpu_rate
    rec.update({"reference_cpu_lower_bound_s": lb, "speedup_vs_reference_lower_bound": lb * 1e3 / rec["wall_ms"],
                "reference_note": "reference MAR = one VE per variable (model.cpp:326-334); bound = n_vars x "
                                  "factor-entries of the width-%d column-sweep PR / measured cpu_baseline rate" % rows})


def merge_sliced(line, sl, world):
    """Put the sliced leg's result into the record: when it ran and is the
    faster of the two schemes measured in this run it becomes the headline
    "mar" (with the instance, the reference bound and the secondary
    instance) and the segment scheme's record moves to "mar_segment"; on
    failure, or when the segment scheme was faster (4 ranks: the projections
    on one GPU are 0.98 s segments against 1.05 s sliced), the segment
    scheme stays the headline and mar["sliced"] holds the leg's record."""
    if "error" in sl or sl.get("wall_ms", float("inf")) >= line["mar"].get("wall_ms", float("inf")):
        line["mar"]["sliced"] = sl
        return
    seg = line["mar"]
    seg.pop("sliced", None)
    head = {"instance": seg["instance"], "scheme": "message-sliced bucket tree over %d ranks "
            "(every message split, one all-to-all per re-slice; DESIGN §6)" % world}
    head.update(sl)
    head["n_gpus"] = world
    for key in ("reference_cpu_lower_bound_s", "reference_note", "secondary"):
        if key in seg:
            head[key] = seg.pop(key)
    seg.pop("speedup_vs_reference_lower_bound", None)
    if "reference_cpu_lower_bound_s" in head:
        head["speedup_vs_reference_lower_bound"] = head["reference_cpu_lower_bound_s"] * 1e3 / head["wall_ms"]
    seg["scheme"] = "chain segments per rank, one all-reduce (DESIGN §6)"
    line["mar"] = head
    line["mar_segment"] = seg


def fp64_bucket(ctx, dev, stream, rank, k=4, w=14, steps=10):
    """The bench bucket in fp64 (the reference's arithmetic; bit-exact against
    it): m(x, S_1..S_w) * f(x, y) -> sum_x, timed with HIP events on the
    launch stream, with an exact spot check against the same sums in torch."""
    import torch
    import bnpp
    S = k ** w
    g = torch.Generator(device=dev).manual_seed(4321 + rank)
    m_t = torch.rand(k * S, generator=g, device=dev, dtype=torch.float64) * 1.5 + 0.5
    f_t = torch.rand(k * k, generator=g, device=dev, dtype=torch.float64) * 1.5 + 0.5
    out = torch.empty(S * k, device=dev, dtype=torch.float64)
    cards = [k] * (w + 2)

    def step():
        bnpp.bucket_eliminate(ctx, bnpp.F64, cards, [m_t.data_ptr(), f_t.data_ptr()], [list(range(w + 1)), [0, w + 1]],
                              0, out.data_ptr(), list(range(1, w + 2)), stream=stream.cuda_stream)
    for _ in range(3):
        step()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for i in range(steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    alg = 8 * (k * S + k * k + S * k)
    gs = torch.Generator(device=dev).manual_seed(77 + rank)
    idx = torch.randint(0, S * k, (512,), generator=gs, device=dev)
    s_i, y_i = idx // k, idx % k
    M, F = m_t.reshape(k, S), f_t.reshape(k, k)
    acc = torch.zeros(512, device=dev, dtype=torch.float64)
    # on the default stream, like idx above (the bucket's stream is idle after
    # the synchronize); indexing on `stream` with indices made on the default
    # stream raced them -- garbage indices, a faulting gather (two ranks on
    # one GPU, round 4)
    for x in range(k):
        acc = acc + M[x, s_i] * F[x, y_i]
    torch.cuda.synchronize(dev)
    traffic = None
    for tpath in sorted(glob.glob(os.path.join(REPO, "profiles", "traffic_r*.json")), reverse=True):
        tj = json.load(open(tpath))
        if tj.get("k") == k and tj.get("w") == w and tj.get("dtype") == "f64":
            traffic = tj.get("hbm_bytes_per_launch")
            break
    return {"workload": "potts-k%d bucket m(x,S_1..S_%d)*f(x,y)->sum_x, f64" % (k, w), "traffic": traffic,
            "factor_entries_per_s": float(k ** (w + 2)) / (kern_ms * 1e-3), "kernel_ms": kern_ms,
            "alg_bytes_per_launch": alg, "achieved_GBps": alg / (kern_ms * 1e-3) / 1e9,
            "frac": alg / (kern_ms * 1e-3) / HBM_PEAK, "spot_check_exact": bool(torch.equal(out[idx], acc))}


def launcher_cmd(n: int, port: int, argv):
    """The command that starts `n` ranks of this script on one node (the
    driver's own launch line for N > 1)."""
    return [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int, argv) -> int:
    """`python bench.py --gpus N` outside a launcher: start N fresh rank
    processes (children, before this process touches the GPU -- no exec) and
    pass their exit status on.  Rank 0's JSON line is relayed to stdout; the
    launcher's and the ranks' other output goes to stderr."""
    env = dict(os.environ)
    env["BNPP_BENCH_CHILD"] = "1"
    # the ranks' stdout is filtered: the JSON record goes to stdout, anything
    # else (gloo's connection notices, for one) to stderr
    p = subprocess.Popen(launcher_cmd(n, free_port(), argv), env=env, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--w", type=int, default=14)
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--cpu-w", type=int, default=10, help="bucket width of the bounded CPU-baseline sample")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-mar", action="store_true")
    ap.add_argument("--no-mar-f64", action="store_true", help="skip the fp64 32x32 MAR (~25 s)")
    ap.add_argument("--no-fp64", action="store_true")
    ap.add_argument("--mar-rows", type=int, default=32)
    ap.add_argument("--mar-cols", type=int, default=32)
    ap.add_argument("--secondary", default="ising12x12.uai",
                    help="reference-runnable MAR instance timed beside the reference's own BN::marginals")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    # N > 1 without a launcher: start the N ranks ourselves (children)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and os.environ.get("BNPP_BENCH_CHILD") != "1":
        sys.exit(self_launch(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started %d rank(s)" % (args.gpus, world))
    # BNPP_BENCH_REHEARSE=1: rehearse the N-rank path with every rank on the
    # visible GPUs round-robin and gloo instead of RCCL (a one-GPU box checks the
    # multi-rank logic this way; its numbers are not a measurement)
    rehearse = os.environ.get("BNPP_BENCH_REHEARSE") == "1"
    # BNPP_BENCH_DRYRUN=1 (CPU test of the launch path): ranks join a gloo
    # world, check its size and print a stub line; no GPU, no engine
    dryrun = os.environ.get("BNPP_BENCH_DRYRUN") == "1"
    backend = None
    if world > 1:
        backend = "gloo" if (rehearse or dryrun) else "nccl"
        if not dryrun:
            if rehearse:
                local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
        # an RCCL error or timeout (the sliced leg's first run on RCCL is on the
        # driver's node) aborts the communicator and raises in the caller --
        # recorded by sliced_mar -- instead of tearing the process down
        # (torch's default, mode 3)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
        dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    if dryrun:
        if world > 1:
            dist.barrier()
        if rank == 0:
            print(json.dumps({"metric": METRIC, "dryrun": True, "n_gpus": world, "world_size": world,
                              "backend": backend}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    import bnpp
    dev = torch.device("cuda", local)
    ctx = bnpp.Context(local)

    dt = bnpp.F32 if args.dtype == "f32" else bnpp.F64
    tdt = torch.float32 if dt == bnpp.F32 else torch.float64
    eb = 4 if dt == bnpp.F32 else 8
    k, w = args.k, args.w
    S = k ** w
    # global bucket: variable 0 = L (card world, the leading split variable),
    # 1 = x, 2..w+1 = S_1..S_w, w+2 = y.  Rank r holds its L = r slice of m and
    # of the output: views with L conditioned, i.e. a local bucket over (x, S, y).
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    m_t = torch.rand(k * S, generator=g, device=dev, dtype=tdt) * 1.5 + 0.5
    f_t = torch.rand(k * k, generator=g, device=dev, dtype=tdt) * 1.5 + 0.5
    out = torch.empty(S * k, device=dev, dtype=tdt)
    cards = [k] * (w + 2)
    scope_m, scope_f = list(range(w + 1)), [0, w + 1]
    out_vars = list(range(1, w + 2))
    stream = torch.cuda.Stream(dev)              # a real (non-null) stream: kernels and events share it
    torch.cuda.synchronize(dev)

    def step():
        bnpp.bucket_eliminate(ctx, dt, cards, [m_t.data_ptr(), f_t.data_ptr()], [scope_m, scope_f], 0,
                              out.data_ptr(), out_vars, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    entries = float(k ** (w + 2))                  # prod(card) over (x, S, y), per rank per step
    value = world * entries * args.steps / elapsed
    alg_bytes = eb * (k * S + k * k + S * k)       # |m| + |f| + |out|
    achieved = alg_bytes / (kern_ms * 1e-3)

    # sanity: checksum of checksums (sum_out = sum_x rowsum(m)_x * rowsum(f)_x)
    want = (m_t.double().reshape(k, S).sum(1) * f_t.double().reshape(k, k).sum(1)).sum().item()
    got = out.double().sum().item()
    ok = abs(got - want) <= (1e-4 if dt == bnpp.F32 else 1e-9) * want
    # exact spot check: out[s*k + y] = ((0 + m[0,s] f[0,y]) + m[1,s] f[1,y]) + ... in the
    # compute dtype, products and sums rounded one at a time like factor.cpp:131-143, 199-205
    gs = torch.Generator(device=dev).manual_seed(99 + rank)
    idx = torch.randint(0, S * k, (512,), generator=gs, device=dev)
    s_i, y_i = idx // k, idx % k
    M, F = m_t.reshape(k, S), f_t.reshape(k, k)
    acc = torch.zeros(512, device=dev, dtype=tdt)
    for x in range(k):
        acc = acc + M[x, s_i] * F[x, y_i]
    spot_ok = bool(torch.equal(out[idx], acc))
    ok = ok and spot_ok

    fp64 = None
    if not args.no_fp64:
        fp64 = fp64_bucket(ctx, dev, stream, rank)
    del m_t, f_t, out, M, F, acc, idx, s_i, y_i
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()

    traffic = None
    # newest profiles/traffic_rNN.json (tools/profile_bench.sh) for this kernel
    for tpath in sorted(glob.glob(os.path.join(REPO, "profiles", "traffic_r*.json")), reverse=True):
        tj = json.load(open(tpath))
        if tj.get("k") == k and tj.get("w") == w and tj.get("dtype") == args.dtype:
            traffic = tj.get("hbm_bytes_per_launch")
            break

    # the reference's CPU path on rank 0's host cores, at every world size (the
    # other ranks wait at the MAR's first barrier meanwhile)
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(k, args.cpu_w, args.cpu_reps)

    # MAR after the bucket and the CPU baseline (see the module docstring: HBM
    # another process freed is cleared in the background for several seconds)
    mar = None
    if not args.no_mar:
        d = dist if world > 1 else None
        mar = mar_wallclock(ctx, rank, world, d, dev, args.mar_rows, args.mar_cols, "f32", True)
        sliced_in = mar.pop("_model")
        reference_bound(mar, cpu["value"] if cpu else None)
        if rank == 0:
            # SURVEY 8(d) C3's reference-runnable MAR: the 12x12 grid (the
            # reference's BN::marginals takes 25-55 s on one core)
            mar["secondary"] = secondary_mar(ctx, args.secondary, not args.no_cpu)
    # the same 32x32 MAR in the reference's precision (fp64, factor.hh:46):
    # split runs of 7 buckets, 32-GiB messages, 3 checkpoint slots -- in the
    # fp32 MAR's cached arena (the same size), as a serving process would run
    # it: freeing that arena first made the fp64 call wait ~6 s for the
    # driver to clear the 240 GB again
    mar_f64 = None
    if not args.no_mar and not args.no_mar_f64:
        d = dist if world > 1 else None
        mar_f64 = mar_wallclock(ctx, rank, world, d, dev, args.mar_rows, args.mar_cols, "f64", True)
        marg64 = mar_f64.pop("_model")[3]
        if mar is not None:
            # every one of the R x C marginals: the fp32 MAR against this
            # independent fp64 one (other plan, slots, kernels) -- the
            # north star's 1e-6 tolerance, at full size
            marg32 = sliced_in[3]
            diff = max(max(abs(a - b) for a, b in zip(marg32[t], marg64[t])) for t in marg64)
            mar["check_vs_fp64"] = {"method": "max |p_fp32 - p_fp64| over every marginal entry", "max_abs_diff": diff,
                                    "tolerance": 1e-6, "ok": diff <= 1e-6}
        reference_bound(mar_f64, cpu["value"] if cpu else None)
        ctx.trim()

    # every check that decides the exit status, before anything can print
    for rec in (mar, mar_f64):
        for key in ("check", "check_vs_fp64"):
            if rec and key in rec and not rec[key]["ok"]:
                ok = False
    if mar and "secondary" in mar and mar["secondary"].get("ok") is False:
        ok = False
    if fp64 is not None and not fp64["spot_check_exact"]:
        ok = False

    line = None
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "factor-entries/s",
            "n_gpus": world,
            "world_size": world,
            "backend": None if world == 1 else ("nccl (RCCL)" if backend == "nccl" else backend),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (U(0.5,2) potentials, seeded)",
            "config": {"workload": "potts-k%d bucket m(x,S_1..S_%d)*f(x,y)->sum_x (BASELINE config 5 restated, "
                                   "SURVEY.md 8(d)); one independent bucket per rank" % (k, w),
                       "k": k, "w": w, "entries_per_gpu_step": entries, "parallelism": "bucket-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
                         "kernel_ms": kern_ms},
            "cpu_baseline": cpu,
            "mar": mar,
            "mar_f64": mar_f64,
            "fp64_bucket": fp64,
            "checksum_ok": ok,
            "spot_check_exact": spot_ok,
        }
    # exactly one JSON line, whichever thread gets there first
    import threading
    print_lock = threading.Lock()
    printed = [False]

    def emit():
        with print_lock:
            if line is not None and not printed[0]:
                print(json.dumps(line), flush=True)
                printed[0] = True

    # From 4 ranks the message-sliced tree MAR also runs
    # (bnpp.dist.sliced_tree_marginals: every message split over the ranks, one
    # all-to-all per re-sliced message -- the north star's scaling MAR, DESIGN
    # §6), and the faster of the two schemes is the headline "mar", the other
    # beside it (merge_sliced).  Two ranks: one xGMI link would carry 7/8 of
    # every re-sliced message, so only the segment scheme runs.
    # BNPP_BENCH_SLICED=0 skips the leg.
    # Its collectives run in process groups with a 120-s timeout and any
    # exception is recorded; a watchdog prints the record with the segment
    # scheme's MAR should the leg not return at all.
    sliced_min = 2 if rehearse else 4
    if mar and world >= sliced_min and world & (world - 1) == 0 and os.environ.get("BNPP_BENCH_SLICED", "1") != "0":
        if line is not None:
            line["mar"]["sliced"] = {"error": "watchdog: the sliced leg did not return"}

        def watchdog():
            if not done.wait(float(os.environ.get("BNPP_BENCH_SLICED_WATCHDOG_S", "300"))):
                emit()
                os._exit(0 if ok else 3)
        done = threading.Event()
        threading.Thread(target=watchdog, daemon=True).start()
        m_, order_, dt_, marg_ = sliced_in
        sl = sliced_mar(ctx, rank, world, dist, dev, m_, order_, dt_, marg_)
        with print_lock:
            done.set()
            if line is not None and not printed[0]:
                merge_sliced(line, sl, world)
        if "error" not in sl and not sl.get("ok", False):
            ok = False                                     # the sliced marginals disagree with the segment scheme
    emit()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
