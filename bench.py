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
import statistics
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
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5", "nb", "sc"], default="c2",
                    help="c2 GL-10D 1 obs (headline, weak-scaling replicas); c3 SLCP 1 obs (box-prior rejection); "
                         "c4 two-moons TSNPE-PFN 5 x 200 (per-round split); "
                         "c5 64 obs sharded over the ranks (strong scaling); nb the reference's own published "
                         "workload (notebooks/benchmark_sample_batched.ipynb: loop vs sample_batched); sc the "
                         "reference's notebooks/sampling_comparison.ipynb (theta 2D / x 50D, 100 sims)")
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
    ap.add_argument("--ia-stress", type=float, default=1.0,
                    help="multiply every item-attention score by this factor (npfn_debug_item_attn_scale): a "
                         "stress run of the first pass's online-softmax fallback; 1 = the model")
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
    thr = n_threads()
    return {
        "value": n_samples / total,
        "value_basis": (f"extrapolated from the timed fits and {rows}-row predicts below to one {n_samples}-sample "
                        "call; the measured end-to-end point is c2_measured (fit-dominated at its small sample "
                        "count)"),
        "unit": "posterior samples/s",
        "cores": thr,
        "cores_note": (f"{thr} oracle worker threads = the job's CPU share (OMP_NUM_THREADS / NPFN_ORACLE_THREADS), "
                       f"not every core of the host: the host shows {os.cpu_count()} logical CPUs "
                       f"({_cpu_model()})"),
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


# notebooks/sampling_comparison.ipynb (reference), cells 9 and 11: seconds for 10 samples of one
# observation / one sample for each of 10 observations (TabPFN_Based_NPE_PFN, theta 2D, x 50D, 100
# simulations; the notebook printed "Device: cpu") -- context, not a target
SC_PUBLISHED_S = {"A_10_samples_1_obs": 8.1098, "B_1_sample_10_obs": 73.9022}


def sc_task():
    """The notebook's model and draws in its RNG order (cells 3, 5, 9, 11): torch.manual_seed(42); A [50, 2],
    b [50]; prior N(0, I2); 100 calibration simulations; one test observation; then 10 more."""
    torch.manual_seed(42)
    A = torch.randn(50, 2)
    b = torch.randn(50)

    def simulator(th):
        return th @ A.T + b + 0.1 * torch.randn(th.shape[0], 50)

    prior = torch.distributions.MultivariateNormal(loc=torch.zeros(2), covariance_matrix=torch.eye(2))
    theta_cal = prior.sample((100,))
    y_cal = simulator(theta_cal)
    y_single = simulator(prior.sample((1,)))
    y_multi = simulator(prior.sample((10,)))
    return theta_cal, y_cal, y_single, y_multi, prior, simulator


def run_sampling_comparison(args, dev):
    """--config sc: the reference's notebooks/sampling_comparison.ipynb on the engine: strategy A =
    sample((N,)) for one observation, strategy B = N calls of sample((1,)), one per observation, for
    N = 10 (the published cells) and the notebook's scaling loop N = 20 / 50 / 100 / 200.  x is
    50-D, so every fit is a tabpfn-sized table under the default ensemble (114 features, 58 tokens)."""
    from npe_pfn import TabPFN_Based_NPE_PFN

    th, y, y1, y10, _, simulator = sc_task()
    prior = torch.distributions.MultivariateNormal(loc=torch.zeros(2, device=dev), covariance_matrix=torch.eye(2, device=dev))
    post = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"device": dev, "random_state": 0,
                                                                     "preprocessing": args.preprocessing})
    post.append_simulations(th.to(dev), y.to(dev))
    y1, y10 = y1.to(dev), y10.to(dev)
    g = torch.Generator().manual_seed(7)
    extra = {n: simulator(torch.randn(n, 2, generator=g)).to(dev) for n in (20, 50, 100, 200)}

    def best_of(fn):
        best = float("inf")
        for _ in range(max(1, args.steps)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best, out

    for _ in range(max(1, args.warmup)):
        post.sample((1,), x=y1)
    rows = {}
    for n, ys in [(10, y10)] + list(extra.items()):
        ta, sa = best_of(lambda: post.sample((n,), x=y1))
        tb, sb = best_of(lambda: torch.stack([post.sample((1,), x=ys[i:i + 1])[0] for i in range(n)]))
        assert sa.shape == (n, 2) and sb.shape == (n, 2) and torch.isfinite(sa).all() and torch.isfinite(sb).all()
        rows[str(n)] = {"A_s": round(ta, 5), "B_s": round(tb, 5), "B_over_A": round(tb / ta, 2)}
    r10 = rows["10"]
    line = {
        "metric": "seconds, sampling_comparison notebook (theta 2D / x 50D, 100 sims): 10 samples of 1 obs",
        "value": r10["A_s"],
        "unit": "s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(r10["A_s"] * 1e3, 3),
        "higher_is_better": False,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic: the notebook's own seeded model and draws (torch.manual_seed(42)); synthetic seeded "
                "TabPFN-v2 weights",
        "config": {"workload": "notebooks/sampling_comparison.ipynb: TabPFN_Based_NPE_PFN, Gaussian prior theta 2D, "
                               "linear simulator x 50D, 100 sims; A = sample((N,)) for 1 obs, B = N x sample((1,)) "
                               f"for N obs; best of {max(1, args.steps)} runs", "preprocessing": args.preprocessing},
        "per_N": rows,
        "published_s": SC_PUBLISHED_S,
        "note": "published_s are the reference notebook's printed seconds at N = 10 (its device line says cpu): "
                "context, not a target",
    }
    print(json.dumps(line), flush=True)


def run_c4(args, dev):
    """--config c4: run_tsnpe_pfn with the demo's two-moons recipe (5 rounds x 200 sims,
    proposal_batch_size 1000, ratio-based support, demo.ipynb:357-364; tsnpe_pfn.py:80-117).
    Wall clock per run and per round, split into proposal sampling (PosteriorSupport rejection:
    prior draws + ratio log-probs), simulator, support threshold (posterior sample of 10 000 +
    ratio log-prob quantile) and, inside those, the classifier's fit and predict and the NPE
    sample() calls.  A second, profiled run gives the classifier engine's kernel table and the
    roofline of its dominant kernel (the 10 000-row train self-attention through k_item_attn)."""
    import npe_pfn.npe_pfn as nmod
    import npe_pfn.support_posterior as sp
    import npe_pfn.tabpfn as tp
    import npe_pfn.tsnpe_pfn as tmod
    from npe_pfn.engine import Engine
    from npe_pfn.tasks import two_moons_prior, two_moons_simulator

    timers, counts = {}, {}
    marks = []
    engines = {"classifier": [], "regressor": []}
    prof_on = {"on": False}

    def wrap(obj, name, key, hook=None):
        orig = getattr(obj, name)

        def w(*a, **k):
            if hook:
                hook(a)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = orig(*a, **k)
            torch.cuda.synchronize()
            timers[key] = timers.get(key, 0.0) + time.perf_counter() - t0
            counts[key] = counts.get(key, 0) + 1
            return r
        setattr(obj, name, w)
        return orig

    def round_mark(_a):
        marks.append(dict(timers))

    def clf_engine(a):
        eng = a[0].engine
        if eng not in engines["classifier"]:
            engines["classifier"].append(eng)
            eng.prof_enable(prof_on["on"])

    def reg_engine(a):
        eng = a[0]._model.engine
        if eng not in engines["regressor"]:
            engines["regressor"].append(eng)
            eng.prof_enable(prof_on["on"])

    saved = [(tmod, "simulate", wrap(tmod, "simulate", "simulate", round_mark)),
             (sp.PosteriorSupport, "__init__", wrap(sp.PosteriorSupport, "__init__", "support_threshold")),
             (sp.PosteriorSupport, "sample", wrap(sp.PosteriorSupport, "sample", "proposal_sampling")),
             (tp.TabPFNClassifier, "fit", wrap(tp.TabPFNClassifier, "fit", "classifier_fit", clf_engine)),
             (tp.TabPFNClassifier, "predict_proba_tensor",
              wrap(tp.TabPFNClassifier, "predict_proba_tensor", "classifier_predict")),
             (nmod.NPE_PFN_Core, "sample", wrap(nmod.NPE_PFN_Core, "sample", "npe_sample", reg_engine)),
             (Engine, "__init__", wrap(Engine, "__init__", "engine_create"))]
    sim_t = {"s": 0.0}

    def simulator(theta):
        t0 = time.perf_counter()
        out = two_moons_simulator(theta)
        sim_t["s"] += time.perf_counter() - t0
        return out

    def run_once(seed):
        timers.clear()
        counts.clear()
        marks.clear()
        sim_t["s"] = 0.0
        torch.manual_seed(seed)
        prior = two_moons_prior()
        x_o = two_moons_simulator(0.5 * torch.ones(1, 2))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        post = tmod.run_tsnpe_pfn(simulator, prior, x_o, num_simulations=1000, num_rounds=5,
                                  proposal_batch_size=1000, regressor_init_kwargs={"device": dev},
                                  classifier_init_kwargs={"device": dev})
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
        assert post._theta_train.shape == (1000, 2)
        return total, post

    try:
        for _ in range(max(1, args.warmup)):
            run_once(0)
        runs = []
        for i in range(max(1, min(args.steps, 3))):
            total, _ = run_once(0)
            runs.append((total, dict(timers), dict(counts), list(marks), sim_t["s"]))
        best = min(runs, key=lambda r: r[0])
        total, tm, cnt, mk, sim_s = best
        bounds = mk + [tm]
        per_round = []
        for r in range(len(mk)):
            a, b = bounds[r], bounds[r + 1]
            d = {k: round((b.get(k, 0.0) - a.get(k, 0.0)) * 1e3, 2) for k in b}
            per_round.append(d)
        # profiled run: the classifier and regressor engines' kernel tables
        prof_on["on"] = True
        engines["classifier"].clear()
        engines["regressor"].clear()
        run_once(0)
        prof = {}
        for kind, engs in engines.items():
            agg = {}
            for eng in engs:
                for e in eng.prof_read():
                    a = agg.setdefault(e["name"], {"name": e["name"], "launches": 0, "ms": 0.0, "flops": 0.0,
                                                  "bytes": 0.0})
                    for key in ("launches", "ms", "flops", "bytes"):
                        a[key] += e[key]
                eng.prof_enable(False)
            prof[kind] = list(agg.values())
    finally:
        for obj, name, orig in saved:
            setattr(obj, name, orig)
    split = {k: round(v * 1e3, 2) for k, v in tm.items()}
    split["simulator_ms"] = round(sim_s * 1e3, 2)

    def table(p):
        return {e["name"]: {"ms": round(e["ms"], 2), "launches": e["launches"],
                            "tflops": round(e["flops"] / (e["ms"] / 1e3) / 1e12, 1) if e["flops"] and e["ms"] else None}
                for e in sorted(p, key=lambda e: -e["ms"])}
    line = {
        "metric": "seconds per run_tsnpe_pfn, Two-Moons TSNPE-PFN 5 rounds x 200 sims",
        "value": round(total, 4),
        "unit": "s",
        "n_gpus": 1,
        "steps": len(runs),
        "warmup": args.warmup,
        "ms_per_step": round(total * 1e3, 2),
        "higher_is_better": False,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic: the demo's two-moons simulator and Uniform(-1, 1)^2 prior (torch.manual_seed(0)); synthetic "
                "seeded TabPFN-v2 regressor / classifier weights",
        "config": {"workload": "run_tsnpe_pfn(two_moons, 5 rounds x 200 sims, proposal_batch_size=1000, ratio_based "
                               "support with 10 000 posterior samples, rejection), demo.ipynb:357-364; best of "
                               f"{len(runs)} runs", "preprocessing": "ensemble (regressor and classifier defaults)"},
        "split_ms": split,
        "calls": cnt,
        "per_round_ms": per_round,
        "classifier_roofline": roofline(prof["classifier"], None) if prof["classifier"] else None,
        "classifier_kernels": table(prof["classifier"]),
        "regressor_kernels": table(prof["regressor"]),
        "note": "split_ms entries nest: support_threshold and proposal_sampling contain npe_sample / classifier_fit / "
                "classifier_predict; simulate contains proposal_sampling and the simulator; per_round_ms[r] runs from "
                "round r's simulate() to the next; the kernel tables come from a separate profiled run",
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
    tr, src = None, None
    if traffic and traffic.get("kernel") == dom["name"]:
        tr = traffic.get("bytes_per_launch")
        # the PMC passes are separate rocprofv3 runs (never inside this process): say which file and
        # tree the bytes come from
        src = traffic.get("source", "profiles/traffic.json (builder's rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)")
    return {
        "bound": "mfma" if mfma else "hbm",
        "kernel": dom["name"],
        "achieved": round(achieved, 2),
        "peak": peak,
        "unit": unit,
        "frac": round(achieved / peak, 4),
        "traffic": tr,
        "traffic_source": src,
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


def rank_identity(dev, world: int, backend: str):
    """N > 1: every rank's device ordinal and PCI bus id, gathered to all ranks; under RCCL
    ("nccl") rank 0 asserts that no two ranks drive the same GPU, so the driver's SCALE record
    proves that N distinct devices ran."""
    import torch.distributed as dist

    p = torch.cuda.get_device_properties(dev)
    mine = {"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "device": dev.index, "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "name": p.name}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    ids = [r["pci_bus_id"] for r in allr]
    if backend == "nccl":
        assert len(set(ids)) == world, f"ranks share a GPU under RCCL: {ids}"
    return {"backend": backend, "world_size": world, "ranks": allr, "distinct_devices": len(set(ids))}


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
    if args.config in ("nb", "sc", "c4"):
        if world > 1:
            raise SystemExit(f"--config {args.config} is a one-GPU workload")
        {"nb": run_notebook, "sc": run_sampling_comparison, "c4": run_c4}[args.config](args, dev)
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

    def timed(steps, fn=None):
        """K steps, each bracketed by a barrier + device synchronize on both sides (SURVEY.md §8d:
        synchronize before starting and after stopping the clock); returns the whole region's
        wall time and every step's, each the max over ranks."""
        fn = fn or step
        per = []
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t_all = time.perf_counter()
        for _ in range(steps):
            if world > 1:
                torch.distributed.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            if world > 1:
                torch.distributed.barrier()
            per.append(time.perf_counter() - t0)
        el = time.perf_counter() - t_all
        if world > 1:
            t = torch.tensor([el] + per, device=dev if torch.distributed.get_backend() == "nccl" else "cpu",
                             dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el, per = float(t[0].item()), [float(v) for v in t[1:].tolist()]
        return el, out, per

    if args.ia_stress != 1.0:
        eng.debug_item_attn_scale(args.ia_stress)
    eng.prof_enable(args.profile_all)
    for _ in range(args.warmup):
        step()
    eng.prof_enable(args.profile_all)
    elapsed, out, step_s = timed(args.steps)   # headline: no per-launch events, fits overlapped
    assert torch.isfinite(out).all(), "non-finite posterior samples"
    eng.prof_read()                            # drop anything recorded so far
    eng.item_attn_fallback(reset=True)
    eng.prof_enable(True)
    prof_steps = max(1, min(args.prof_steps, args.steps))
    if world > 1:
        from npe_pfn.distributed import phase_timing

        phase_timing(True)
    if world > 1:
        from npe_pfn.distributed import collective_stats

        collective_stats(reset=True)           # count the profiled pass's collectives only
    elapsed_prof, _, _ = timed(prof_steps)     # roofline / kernel table pass (fits in order)
    eng.prof_enable(False)
    prof = eng.prof_read()
    ia_fb = eng.item_attn_fallback(reset=True)
    if args.ia_stress != 1.0:
        eng.debug_item_attn_scale(1.0)
    per_rank = None
    if world > 1:
        per_rank = per_rank_split(prof, prof_steps, elapsed_prof, rank, world)
        from npe_pfn.distributed import collective_stats

        coll = collective_stats()
        per_rank["collective_bytes_per_step"] = {k: {"calls": v["calls"] / prof_steps, "bytes": v["bytes"] / prof_steps}
                                                 for k, v in coll.items()}
        per_rank["identity"] = rank_identity(dev, world, torch.distributed.get_backend())
    alt_modes = None
    if world > 1 and mode == "ep":
        # the north_star form beside the default EP line (BASELINE.json north_star: replicated fit,
        # row shards, ONE gather at the end): the same call with --mode rows, timed the same way
        # in the same processes, its collectives counted, its draws compared with the EP call's
        from npe_pfn.distributed import collective_stats

        def step_rows():
            return sample_rows_sharded(post, x_o, (N,))

        for _ in range(max(1, args.warmup)):
            step_rows()
        collective_stats(reset=True)
        _, _, rows_s = timed(args.steps, step_rows)
        coll_rows = collective_stats()
        rows_med = statistics.median(rows_s)
        # one more call of each form from the same Philox counter: the draws must be equal
        reg = post._model
        c0 = reg.sample_counter
        out_ep = step()
        reg.sample_counter = c0
        out_rows = step_rows()
        alt_modes = {"rows": {
            "value": round(N / rows_med, 2), "ms_per_step": round(rows_med * 1e3, 3),
            "parallelism": f"rows{world} (row shards, replicated fit, one all_gather at the end)",
            "step_ms": [round(v * 1e3, 3) for v in rows_s],
            "collective_bytes_per_step": {k: {"calls": v["calls"] / args.steps, "bytes": v["bytes"] / args.steps}
                                          for k, v in coll_rows.items()},
            "draws_equal_to_ep": bool(torch.equal(out_rows, out_ep)),
        }}
    # headline: the median timed call (SURVEY.md §8d / BASELINE.md: "the median of 5 runs"; with
    # the default --steps the median of >= 5); the mean over the K calls is reported beside it
    med_s = statistics.median(step_s)
    value = units / med_s
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
        "ms_per_step": round(med_s * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "bf16",
        "data": data + "; synthetic seeded weights of the TabPFN-v2 regressor architecture (no checkpoint "
                       "available offline)",
        "config": {"workload": workload, "global_batch": units, "seq_len": n_sims, "parallelism": par,
                   "preprocessing": args.preprocessing},
        "roofline": roofline(prof, traffic),
        "timing": {"statistic": f"median of the {args.steps} timed calls (each bracketed by barrier + synchronize)",
                   "value_mean": round(units * args.steps / elapsed, 2),
                   "ms_per_step_mean": round(elapsed / args.steps * 1e3, 3),
                   "step_ms": [round(v * 1e3, 3) for v in step_s], "region_s": round(elapsed, 4)},
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
    if alt_modes is not None:
        line["alt_modes"] = alt_modes
    line["kernels"] = {e["name"]: {"ms_per_step": round(e["ms"] / prof_steps, 2), "launches": e["launches"],
                                   "tflops": round(e["flops"] / (e["ms"] / 1e3) / 1e12, 1) if e["flops"] else None,
                                   "gbs": round(e["bytes"] / (e["ms"] / 1e3) / 1e9, 1)}
                       for e in sorted(prof, key=lambda e: -e["ms"])}
    if "k_item_attn" in line["kernels"]:
        # share of query rows / blocks whose reference-free first pass failed its range check and
        # took the online-softmax pass (device counters over the profiled pass)
        line["kernels"]["k_item_attn"]["fallback_frac"] = round(ia_fb["fallback_frac"], 6)
        line["kernels"]["k_item_attn"]["block_fallback_frac"] = round(ia_fb["block_fallback_frac"], 6)
    if args.ia_stress != 1.0:
        line["config"]["ia_stress"] = args.ia_stress
        line["data"] += (f"; STRESS RUN: every item-attention score x{args.ia_stress} (fallback cost measurement, "
                         "not the model)")
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
