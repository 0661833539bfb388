#!/usr/bin/env python
"""Posterior samples/s on Gaussian-linear 10D with 1000 simulations (BASELINE.json metric).

One step = one ``TabPFN_Based_NPE_PFN.sample((10000,), x=x_o)`` call, i.e. the
reference's timed call: std-Euclidean context filter, the
accept/reject loop and all 10 autoregressive dimensions, each with its fit
(train-side forward of the 1000-row context) and its predict over the 10 000
query rows.  Inputs are resident in HBM before the timed region.

Multi-GPU (one rank per GPU over RCCL; ``--gpus N`` without torchrun re-launches itself
under ``torch.distributed.run`` before touching the GPU):

* ``--mode ep`` (default at N > 1, strong scaling): the SAME single ``sample((10000,))``
  call split by estimator (npe_pfn.distributed.sample_estimator_parallel): every rank
  fits and forwards E/N estimators, one all_to_all of target tokens and one all_gather
  of the sampled column per AR step; identical draws to the 1-GPU call.
  ``value`` = 10 000 samples x steps / max-over-ranks wall time;
* ``--mode rows``: the row split with the fit replicated per rank (strong);
* ``--mode replicas``: every rank its own 10 000 draws (weak; labelled as such).

The headline ``value`` comes from a timed pass with per-launch profiling OFF; the
roofline object and the per-kernel table come from a second pass of the same
workload with HIP events around every engine launch (npfn_prof_*; the AR fits then run
in order on the main stream, so each event pair times its launch alone); FLOPs and bytes
are algorithmic.  ``--profile-all`` profiles the warmup and headline passes
too: the form the rocprofv3 kernel-stats run uses, so its durations match the live ones.  ``cpu_baseline`` runs the CPU oracle (numpy
restatement, oracle/) on rank 0 at N=1 on a bounded sample (see its "sample").
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "npe-pfn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--mode", choices=["auto", "ep", "rows", "replicas"], default="auto",
                    help="multi-GPU split of c2/c3 (auto: ep when the world size divides n_estimators, else rows)")
    ap.add_argument("--prof-steps", type=int, default=5, help="steps of the profiled pass (roofline, kernels)")
    ap.add_argument("--profile-all", action="store_true",
                    help="profile every pass (the AR fits then run in order on the main stream): for the "
                         "rocprofv3 kernel-stats run, whose per-kernel durations must match the profiled pass's")
    ap.add_argument("--config", choices=["c2", "c3", "c5", "nb"], default="c2",
                    help="c2 GL-10D 1 obs (headline, weak-scaling replicas); c3 SLCP 1 obs (box-prior rejection); "
                         "c5 64 obs sharded over the ranks (strong scaling); nb the reference's own published "
                         "workload (notebooks/benchmark_sample_batched.ipynb: loop vs sample_batched)")
    ap.add_argument("--obs", type=int, default=64, help="observations for --config c5")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples", type=int, default=10_000)
    ap.add_argument("--sims", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--preprocessing", choices=["ensemble", "none", "quantile", "quantile+power"], default="ensemble",
                    help="per-estimator preprocessing (Engine.set_preprocessing); default: tabpfn's regressor ensemble")
    ap.add_argument("--cpu-rows", type=int, default=256, help="query rows per step in the CPU-baseline sample")
    ap.add_argument("--cpu-measured", type=int, default=64,
                    help="samples of the end-to-end c2 oracle sample() measured beside the extrapolation (0: skip)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes of the dominant kernel from a rocprofv3 --pmc run")
    return ap.parse_args()


def gl_task(D: int, n: int, seed: int = 0):
    """sbibm Gaussian-linear; npe_pfn.tasks.gaussian_linear_task."""
    from npe_pfn.tasks import gaussian_linear_task

    return gaussian_linear_task(D, n, seed)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_c1_end_to_end(weights, cfg):
    """Measured (not extrapolated): the oracle driven through NPE_PFN_Core's reference loop
    (fit / predict / criterion.sample per dimension) for config c1 -- GL-2D, 200
    simulations, sample((1000,))."""
    from npe_pfn import NPE_PFN_Core
    from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task
    from oracle.tabpfn_oracle import OracleRegressor

    theta, x, x_o = gaussian_linear_task(2, 200, seed=0)
    core = NPE_PFN_Core(prior=gaussian_linear_prior(2))
    core._model = OracleRegressor(cfg.n_estimators, cfg.softmax_temperature, random_state=0, weights=weights)
    core.append_simulations(theta, x)
    t0 = time.perf_counter()
    s = core.sample((1000,), x=x_o)
    dt = time.perf_counter() - t0
    assert s.shape == (1000, 2) and torch.isfinite(s).all()
    return {"value": round(1000 / dt, 2), "seconds": round(dt, 2),
            "workload": "c1: GL-2D, 200 sims, NPE_PFN_Core.sample((1000,)) end to end (2 AR dims, 8 estimators)"}


def cpu_c2_end_to_end(weights, cfg, theta, x, x_o, n: int, preprocessing: str):
    """Measured (not extrapolated): the oracle driven through TabPFN_Based_NPE_PFN's reference
    loop (std-Euclid filter, accept/reject, fit / predict / criterion.sample per dimension) on
    the c2 workload itself -- GL-10D, 1000 simulations -- for sample((n,))."""
    from npe_pfn import TabPFN_Based_NPE_PFN
    from npe_pfn.tasks import gaussian_linear_prior
    from oracle.tabpfn_oracle import OracleRegressor

    post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(theta.shape[1]))
    post._model = OracleRegressor(cfg.n_estimators, cfg.softmax_temperature, random_state=0, weights=weights,
                                  preprocessing=preprocessing)
    post.append_simulations(theta.cpu(), x.cpu())
    t0 = time.perf_counter()
    s = post.sample((n,), x=x_o.cpu())
    dt = time.perf_counter() - t0
    assert s.shape == (n, theta.shape[1]) and torch.isfinite(s).all()
    return {"value": round(n / dt, 3), "seconds": round(dt, 2), "samples": n,
            "workload": f"c2: GL-{theta.shape[1]}D, {x.shape[0]} sims, TabPFN_Based_NPE_PFN.sample(({n},)) end to end "
                        f"through the oracle ({preprocessing} preprocessing, 8 estimators)"}


def cpu_baseline(theta, x, x_o, n_samples: int, rows: int, preprocessing: str = "none", measured_n: int = 64):
    """Oracle (numpy, multi-threaded) on a bounded sample of the same workload.

    Timed: the fit on the full context + predict of `rows` query rows at the
    first and last autoregressive step.  Pipeline time for n_samples draws is
    sum_k [fit_k + n_samples/rows * predict_k], with both terms interpolated
    linearly between the first and last step (their cost is linear in the
    step's column count).  Next to it, config c1 is measured end to end.
    """
    from npe_pfn.weights import ModelConfig, synthetic_weights
    from oracle.tabpfn_oracle import OracleTabPFN, n_threads

    cfg = ModelConfig()
    w = synthetic_weights(cfg, seed=0)
    pre = {"none": 0, "quantile": 1, "quantile+power": 2, "ensemble": 3}[preprocessing]
    m = OracleTabPFN(w, cfg.n_estimators, cfg.softmax_temperature, seed=0, preprocessing=pre)
    th, xx, xo = theta.cpu().numpy(), x.cpu().numpy(), x_o.cpu().numpy()
    dx, D = xx.shape[1], th.shape[1]
    joint = np.concatenate([xx, th], 1)
    rng = np.random.default_rng(0)
    t_fit, t_pred = [], []
    for k in (0, D - 1):
        F = dx + k
        t0 = time.perf_counter()
        m.fit(joint[:, :F], joint[:, F])
        t1 = time.perf_counter()
        q = np.concatenate([np.repeat(xo, rows, 0), rng.normal(0, 0.3, (rows, k)).astype(np.float32)], 1)
        m.predict_probs(q)
        t2 = time.perf_counter()
        t_fit.append(t1 - t0)
        t_pred.append(t2 - t1)
    def model_seconds(n):
        return sum((t_fit[0] + (t_fit[1] - t_fit[0]) * k / max(D - 1, 1))
                   + n / rows * (t_pred[0] + (t_pred[1] - t_pred[0]) * k / max(D - 1, 1)) for k in range(D))

    total = model_seconds(n_samples)
    meas = cpu_c2_end_to_end(w, cfg, theta, x, x_o, measured_n, preprocessing) if measured_n > 0 else None
    if meas is not None:
        pred = model_seconds(measured_n)
        meas["extrapolation_model_seconds"] = round(pred, 2)
        meas["model_vs_measured"] = round(pred / meas["seconds"], 3)
    return {
        "value": n_samples / total,
        "unit": "posterior samples/s",
        "cores": n_threads(),
        "cpu_model": _cpu_model(),
        "kind": "port",
        "sample": (f"oracle fit (n={xx.shape[0]}) + predict of {rows} rows at AR steps 0 and {D - 1} "
                   f"({sum(t_fit) + sum(t_pred):.1f} s measured); {n_samples}-sample sample() time "
                   f"extrapolated over {D} steps = {total:.0f} s"),
        "c1_measured": cpu_c1_end_to_end(w, cfg),
        "c2_measured": meas,
    }


# notebooks/benchmark_sample_batched.ipynb (reference), cell 8 output: seconds for n_obs
# observations x 100 samples, NPE_PFN_Core on a theta 3D / x 10D linear-Gaussian model with 1000
# simulations; hardware not stated in the notebook -- context, not a target
NB_PUBLISHED_S = {5: (8.2832, 2.6127), 10: (16.2372, 3.5990), 20: (33.8342, 6.3405), 50: (87.1265, 12.3774)}


def notebook_task():
    """The notebook's model and draws, in its own RNG order (cells 1-4, 7, 8): torch.manual_seed(42);
    A [10, 3], b [10] ~ randn; prior N(0, I3); 1000 training simulations; a 2-row warm-up x; then per
    n_obs in (5, 10, 20, 50) theta_test ~ prior, x_test = simulator(theta_test)."""
    torch.manual_seed(42)
    np.random.seed(42)
    torch.manual_seed(42)
    A = torch.randn(10, 3)
    b = torch.randn(10)

    def simulator(th):
        return th @ A.T + b + 0.1 * torch.randn(th.shape[0], 10)

    prior = torch.distributions.MultivariateNormal(loc=torch.zeros(3), covariance_matrix=torch.eye(3))
    theta_train = prior.sample((1000,))
    x_train = simulator(theta_train)
    x_warm = torch.randn(2, 10)
    tests = {}
    for n_obs in (5, 10, 20, 50):
        th = prior.sample((n_obs,))
        tests[n_obs] = simulator(th)
    return prior, theta_train, x_train, x_warm, tests


def run_notebook(args, dev):
    """--config nb: the notebook's timing loop on the engine (loop of sample() per observation vs
    one sample_batched()), the notebook's published seconds printed beside the measured ones."""
    from npe_pfn import NPE_PFN_Core

    prior, th_tr, x_tr, x_warm, tests = notebook_task()
    prior_dev = torch.distributions.MultivariateNormal(loc=torch.zeros(3, device=dev),
                                                       covariance_matrix=torch.eye(3, device=dev))
    model = NPE_PFN_Core(prior=prior_dev, regressor_init_kwargs={"device": dev, "random_state": 0,
                                                                   "preprocessing": args.preprocessing})
    model.append_simulations(th_tr.to(dev), x_tr.to(dev))
    n = 100

    def loop(xo):
        return torch.stack([model.sample((n,), x=xo[i:i + 1]) for i in range(xo.shape[0])])

    def batched(xo):
        return model.sample_batched(x=xo, sample_shape=(n,))

    xw = x_warm.to(dev)
    for _ in range(max(1, args.warmup)):
        loop(xw)
        batched(xw)
    rows = {}
    for n_obs, xt in tests.items():
        xt = xt.to(dev)
        t = {}
        for name, fn in (("loop", loop), ("batched", batched)):
            best = float("inf")
            for _ in range(max(1, args.steps)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = fn(xt)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            assert out.shape == (n_obs, n, 3) and torch.isfinite(out).all()
            t[name] = best
        pl, pb = NB_PUBLISHED_S[n_obs]
        rows[str(n_obs)] = {"loop_s": round(t["loop"], 4), "batched_s": round(t["batched"], 4),
                            "samples_per_s_batched": round(n_obs * n / t["batched"], 1),
                            "notebook_loop_s": pl, "notebook_batched_s": pb}
    big = rows["50"]
    line = {
        "metric": "posterior samples/sec, notebook linear-Gaussian theta3/x10, 1000 sims, 50 obs x 100 samples, "
                  "sample_batched",
        "value": big["samples_per_s_batched"],
        "unit": "posterior samples/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(big["batched_s"] * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic: the notebook's own seeded model and draws (torch.manual_seed(42)); synthetic seeded "
                "TabPFN-v2 weights",
        "config": {"workload": "notebooks/benchmark_sample_batched.ipynb: NPE_PFN_Core, theta 3D / x 10D, 1000 sims, "
                               "n_obs in 5/10/20/50 x 100 samples, loop of sample() vs sample_batched(); best of "
                               f"{max(1, args.steps)} timed runs each", "preprocessing": args.preprocessing},
        "per_n_obs": rows,
        "note": "notebook_*_s are the reference notebook's published seconds (cell 8; hardware not stated): "
                "context, not a target",
    }
    print(json.dumps(line), flush=True)


def roofline(prof, traffic):
    dom = max(prof, key=lambda e: e["ms"])
    sec = dom["ms"] / 1e3
    # the bound is the roof the kernel sits closer to (flop-heavy kernels: the MFMA peak)
    mfma = dom["flops"] / sec / 1e12 / BF16_PEAK_TFLOPS >= dom["bytes"] / sec / 1e9 / HBM_PEAK_GBS
    if mfma:
        achieved = dom["flops"] / sec / 1e12
        peak, unit = BF16_PEAK_TFLOPS, "TFLOP/s"
    else:
        achieved = dom["bytes"] / sec / 1e9
        peak, unit = HBM_PEAK_GBS, "GB/s"
    tr = None
    if traffic and traffic.get("kernel") == dom["name"]:
        tr = traffic.get("bytes_per_launch")
    return {
        "bound": "mfma" if mfma else "hbm",
        "kernel": dom["name"],
        "achieved": round(achieved, 2),
        "peak": peak,
        "unit": unit,
        "frac": round(achieved / peak, 4),
        "traffic": tr,
        "avg_launch_us": round(dom["ms"] * 1e3 / dom["launches"], 2),
        "launches": dom["launches"],
        "algorithmic_per_launch": (dom["flops"] if mfma else dom["bytes"]) / dom["launches"],
        "time_share": round(dom["ms"] / sum(e["ms"] for e in prof), 3),
    }


def per_rank_split(prof, steps: int, elapsed: float, rank: int, world: int):
    """N > 1: every rank's split of one profiled step (ms) -- compute (fits + test-side forwards),
    exchange (all_to_all of target tokens), head (decoder + mix + sample), gather (all_gather of the
    sampled columns) from npe_pfn.distributed's phase events, and the engine's kernel time -- gathered
    to rank 0, with the max over ranks of each field."""
    import torch.distributed as dist
    from npe_pfn.distributed import phase_timing, phase_timing_read

    ph = phase_timing_read()
    phase_timing(False)
    mine = {"rank": rank, "wall_ms": round(elapsed / steps * 1e3, 3),
            "kernel_ms": round(sum(e["ms"] for e in prof) / steps, 3)}
    for p in ("compute", "exchange", "head", "gather"):
        mine[p + "_ms"] = round(ph[p] / steps, 3)
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    keys = [k for k in mine if k.endswith("_ms")]
    return {"ranks": allr, "max": {k: max(r[k] for r in allr) for k in keys},
            "note": "ms per profiled step (fits in order on the main stream, per-launch events on)"}


def relaunch_distributed(n: int) -> int:
    """``--gpus N`` outside torchrun: run this script under torch.distributed.run with N ranks
    (a child process, started before this process touches the GPU) and return its exit code."""
    import subprocess

    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args.gpus))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using the launcher's {world}", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # NPFN_DIST_BACKEND=gloo: CPU-collective rehearsal of the multi-GPU path (ranks may share
        # one GPU); the default is RCCL ("nccl"), one rank per GPU
        backend = os.environ.get("NPFN_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.config == "nb":
        if world > 1:
            raise SystemExit("--config nb is a one-GPU workload")
        run_notebook(args, dev)
        return

    from npe_pfn import NPE_PFN_Core, TabPFN_Based_NPE_PFN
    from npe_pfn.distributed import (ep_layout, sample_batched_sharded, sample_estimator_parallel, sample_replicas,
                                     sample_rows_sharded)
    from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task, slcp_prior, slcp_task
    from npe_pfn.weights import ModelConfig

    n_sims, N = args.sims, args.samples
    if args.config == "c3":
        theta_c, x_c, xo_c = slcp_task(n_sims, seed=0)
        prior = slcp_prior(device=dev)
    else:
        theta_c, x_c, xo_c = gaussian_linear_task(args.dim, n_sims, seed=0)
        prior = gaussian_linear_prior(args.dim, device=dev)
    D = theta_c.shape[1]
    theta, x, x_o = theta_c.to(dev), x_c.to(dev), xo_c.to(dev)
    mode = args.mode
    if args.config == "c5":
        # one shared context for all observations (reference sample_batched, npe_pfn.py:310-410);
        # observations sharded over the ranks, same random_state everywhere (global Philox rows)
        post = NPE_PFN_Core(prior=prior, regressor_init_kwargs={"random_state": 0, "device": dev,
                                                                  "preprocessing": args.preprocessing})
        post.append_simulations(theta, x)
        x_obs = gaussian_linear_task(args.dim, args.obs, seed=123)[1].to(dev)
        units, scaling, mode = args.obs * N, "strong", "observations"

        def step():
            return sample_batched_sharded(post, x_obs, (N,))
    else:
        if mode == "auto":
            mode = "ep" if world > 1 and ModelConfig().n_estimators % world == 0 else ("rows" if world > 1 else "single")
        seed = rank if mode == "replicas" else 0
        post = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": seed, "device": dev,
                                                                          "preprocessing": args.preprocessing})
        post.append_simulations(theta, x)
        if mode == "replicas":
            units, scaling = world * N, "weak"

            def step():
                return sample_replicas(post, x_o, N)
        elif mode == "ep":
            units, scaling = N, "strong"
            E = ModelConfig().n_estimators
            # balanced EP groups: with the ensemble, a strided set must hold both halves of the
            # ensemble (their estimators differ ~2x in token count), so at most E / 2 ranks per group
            ep_g, ep_rows = ep_layout(world, E, max_ep=E // 2 if args.preprocessing == "ensemble" else E)

            def step():
                return sample_estimator_parallel(post, x_o, (N,), ep_size=ep_g)
        elif mode == "rows":
            units, scaling = N, "strong"

            def step():
                return sample_rows_sharded(post, x_o, (N,))
        else:
            units, scaling = N, "strong"

            def step():
                return post.sample((N,), x=x_o)
    eng = post._model.engine

    def timed(steps):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev if torch.distributed.get_backend() == "nccl" else "cpu",
                             dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        return el, out

    eng.prof_enable(args.profile_all)
    for _ in range(args.warmup):
        step()
    eng.prof_enable(args.profile_all)
    elapsed, out = timed(args.steps)           # headline: no per-launch events, fits overlapped
    assert torch.isfinite(out).all(), "non-finite posterior samples"
    eng.prof_read()                            # drop anything recorded so far
    eng.prof_enable(True)
    prof_steps = max(1, min(args.prof_steps, args.steps))
    if world > 1:
        from npe_pfn.distributed import phase_timing

        phase_timing(True)
    elapsed_prof, _ = timed(prof_steps)        # roofline / kernel table pass (fits in order)
    eng.prof_enable(False)
    prof = eng.prof_read()
    per_rank = None
    if world > 1:
        per_rank = per_rank_split(prof, prof_steps, elapsed_prof, rank, world)
    value = units * args.steps / elapsed
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            traffic = json.load(f)
    if args.config == "c2":
        metric = f"posterior samples/sec, Gaussian-linear {D}D, {n_sims} sims"
        per = "per GPU" if mode == "replicas" else "in one sample() call"
        workload = (f"GL-{D}D, {n_sims} sims, {N} posterior samples {per} via TabPFN_Based_NPE_PFN.sample "
                    f"(std-euclid filter, {D} AR dims, 8 estimators)")
        data = "synthetic (sbibm Gaussian-linear simulator, seeded)"
    elif args.config == "c3":
        metric = f"posterior samples/sec, SLCP 5D/8 obs, {n_sims} sims"
        per = "per GPU" if mode == "replicas" else "in one sample() call"
        workload = (f"SLCP, {n_sims} sims, {N} posterior samples {per} via TabPFN_Based_NPE_PFN.sample "
                    "(box prior U(-3,3)^5 with accept/reject, 5 AR dims, 8 estimators)")
        data = "synthetic (sbibm SLCP simulator, seeded)"
    else:
        metric = f"posterior samples/sec, Gaussian-linear {D}D, {n_sims} sims, {args.obs} observations"
        workload = (f"GL-{D}D, {n_sims} sims, {args.obs} observations x {N} samples via sample_batched, "
                    f"observations sharded over {world} GPU(s)")
        data = "synthetic (sbibm Gaussian-linear simulator, seeded)"
    ep_label = (f"ep{ep_g} (estimator-parallel, strided estimator sets, one sample() call)" if mode == "ep" and
                ep_rows == 1 else f"ep{ep_g}x{ep_rows} (estimator-parallel groups of {ep_g} ranks x {ep_rows} row "
                                  f"groups, one sample() call)" if mode == "ep" else "")
    par = {"single": "dp1", "ep": ep_label,
           "rows": f"rows{world} (row shards, replicated fit)", "replicas": f"dp{world} (weak replicas)",
           "observations": f"obs{world} (observation shards)"}[mode]
    line = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "posterior samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "bf16",
        "data": data + "; synthetic seeded weights of the TabPFN-v2 regressor architecture (no checkpoint "
                       "available offline)",
        "config": {"workload": workload, "global_batch": units, "seq_len": n_sims, "parallelism": par,
                   "preprocessing": args.preprocessing},
        "roofline": roofline(prof, traffic),
    }
    line["step_roofline"] = {
        "algorithmic_tflop_per_step": round(sum(e["flops"] for e in prof) / prof_steps / 1e12, 3),
        "achieved_tflops": round(sum(e["flops"] for e in prof) / elapsed_prof / 1e12, 2),
        "kernel_time_frac": round(sum(e["ms"] for e in prof) / 1e3 / elapsed_prof, 3),
        "ms_per_step_profiled": round(elapsed_prof / prof_steps * 1e3, 3),
        "profiled_steps": prof_steps,
        "rank": rank,
    }
    if per_rank is not None:
        line["per_rank"] = per_rank
    line["kernels"] = {e["name"]: {"ms_per_step": round(e["ms"] / prof_steps, 2), "launches": e["launches"],
                                   "tflops": round(e["flops"] / (e["ms"] / 1e3) / 1e12, 1) if e["flops"] else None,
                                   "gbs": round(e["bytes"] / (e["ms"] / 1e3) / 1e9, 1)}
                       for e in sorted(prof, key=lambda e: -e["ms"])}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        line["cpu_baseline"] = cpu_baseline(theta_c, x_c, xo_c, N, args.cpu_rows, args.preprocessing,
                                            args.cpu_measured)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
