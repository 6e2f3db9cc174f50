"""bench.py — sampled molecules/sec for the equivariant-CNF sample path (BASELINE.json `metric`).

Workloads (BASELINE.json configs):
  * N = 1 (configs[1], the headline): LJ13 (N = 13, D = 3, lj13.yaml network), batch 1024, fixed-step ODE with
    NFE = 100 (Euler, dt = 0.01), synthetic inputs (x0 from the zero-CoM base with a seeded
    draw) and flax-default random-init weights of the lj13 architecture.
  * N > 1 (configs[4]): LJ13 global batch 65536 sharded contiguously over the N ranks (65536 / N molecules per GPU,
    one process per GPU, RCCL), plus the eval leg of setup_training.py:166-185: sample_and_log_prob_cnf (Hutchinson,
    Euler NFE = 100) -> LJ13 target log-density -> log_w -> reverse / forward ESS, reduced over RCCL (one MAX and one
    SUM all-reduce).  Noise is one seeded global draw, so every molecule's result is independent of N.

One "step" = one full sample of the rank's shard: x0 (resident in HBM) -> 100 EGNN evaluations -> x1, i.e. one
ecnf_integrate launch.  The timing is the max over ranks, bracketed by barriers and device syncs.

Launch: `python bench.py --gpus N` with WORLD_SIZE unset starts the N rank processes itself (torch.distributed.run as a
CHILD process, before this process touches the GPU) and exits with its status; under torchrun it is one rank.

Extra fields: "roofline" (dominant kernel = integrate_kernel, MFMA bound: algorithmic fp32 FLOPs per launch /
average launch time from HIP events on the launch stream, against the ceiling of the kernel's instruction mix —
GEMM FLOPs at the split-fp16 rate, vector FLOPs at the fp32 rate; see roofline_peak), "matmul" (which arithmetic the
GEMMs run, and the strict-fp32 kernels' time on the same workload), "logprob" (the eval leg, at every N: the
Hutchinson divergence kernel's time and TFLOP/s), "train" (the flow-matching training step at lj13.yaml's batch 64),
"ref_sampling_latency" (the reference's own timing script: one QM9 molecule per adaptive sample_cnf call) and
"cpu_baseline" (a
torch-CPU fp32 batched restatement of the same Euler solve on a bounded sample, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ecnf-baseline-neurips-2023_amd"))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3    # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md, chip-level parameters)
PEAK_16BIT_MFMA_TFLOPS = 2516.6  # MI355X dense BF16 = FP16 matrix peak: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz
SPLIT_TERMS = {"split_f16": 3, "split_bf16": 6}   # 16-bit cross terms per fp32 product (chain_split.hpp)
GLOBAL_BATCH_MULTI = 65536       # BASELINE.json configs[4]


def flops_per_eval(cfg) -> float:
    """Dense-contraction FLOPs of one EGNN evaluation of one molecule with the phi_e layer-1 per-node
    factorisation: F = K [2N(H+T)H + 4NHM + 3EM + 2E(L-1)M^2 + 2ELM^2 + 4EM
    + 2N((M+H)M + (L-1)M^2 + MH)]."""
    N, H, T, M, L, K = cfg.n_nodes, cfg.hidden, cfg.time_embedding_dim, cfg.mlp_width, cfg.mlp_depth, cfg.n_blocks
    E = N * (N - 1)
    return K * (2 * N * (H + T) * H + 4 * N * H * M + 3 * E * M + 2 * E * (L - 1) * M * M + 2 * E * L * M * M
                + 4 * E * M + 2 * N * ((M + H) * M + (L - 1) * M * M + M * H))


def dead_flops_per_eval(cfg) -> float:
    """FLOPs of flops_per_eval that no output depends on: the last block's h update (gate dot 2EM and phi_h), since
    the field is x_K - x_c - mean(x) (egnn.py:176-188).  jit (XLA dead-code elimination) drops them in the reference
    and the kernel skips them, so the roofline counts live FLOPs only."""
    N, H, M, L = cfg.n_nodes, cfg.hidden, cfg.mlp_width, cfg.mlp_depth
    E = N * (N - 1)
    return 2 * E * M + 2 * N * ((M + H) * M + (L - 1) * M * M + M * H)


def live_flops_per_eval(cfg) -> float:
    return flops_per_eval(cfg) - dead_flops_per_eval(cfg)


def pair_tiles_active(cfg, chain_mode: str) -> bool:
    """Block-1 pair tiles (egnn_eval.hpp PairPlan13; set in ecnf_hip.hip ecnf_create): one node feature, 13 atoms,
    the M = 128 split primal kernels."""
    return chain_mode in SPLIT_TERMS and cfg.n_features == 1 and cfg.n_nodes == 13 and cfg.mlp_width == 128


def executed_flops_per_eval(cfg, chain_mode: str) -> float:
    """live_flops_per_eval as the kernel executes it: with pair tiles, block 1's edge work (layer-1 assembly, the phi_e
    and phi_x chains, the gate and phi_x-output dots) runs once per unordered pair, half the edges (m_ij = m_ji there)."""
    F = live_flops_per_eval(cfg)
    if not pair_tiles_active(cfg, chain_mode):
        return F
    N, M, L = cfg.n_nodes, cfg.mlp_width, cfg.mlp_depth
    E = N * (N - 1)
    edge_block = 3 * E * M + 2 * E * (L - 1) * M * M + 2 * E * L * M * M + 4 * E * M
    return F - edge_block / 2


def vector_flops_per_eval(cfg) -> float:
    """The part of live_flops_per_eval that is not a GEMM (runs on the fp32 VALU): phi_e layer-1 assembly (3EM), the
    phi_x-output dot product (2EM) and the gate dot product (2EM, every block but the last)."""
    N, M, K = cfg.n_nodes, cfg.mlp_width, cfg.n_blocks
    E = N * (N - 1)
    return K * (3 * E * M + 4 * E * M) - 2 * E * M


def roofline_peak(cfg, chain_mode: str) -> float:
    """Ceiling (TFLOP/s of algorithmic fp32 FLOPs) for this kernel's instruction mix.  Split modes run every GEMM
    (edge chain and node GEMMs) on the 16-bit matrix cores at (dense 16-bit peak / cross terms) and the vector
    FLOPs at the fp32 rate: peak = F / (F_gemm / P_split + F_vec / P_fp32); fp32_mfma: the fp32 MFMA peak."""
    F = live_flops_per_eval(cfg)
    if chain_mode not in SPLIT_TERMS:
        return PEAK_FP32_MFMA_TFLOPS
    Fv = vector_flops_per_eval(cfg)
    p_split = PEAK_16BIT_MFMA_TFLOPS / SPLIT_TERMS[chain_mode]
    return F / ((F - Fv) / p_split + Fv / PEAK_FP32_MFMA_TFLOPS)


PMC_PASSES = (("FETCH_SIZE", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES"), ("WRITE_SIZE",))
N_XCD, N_SIMD = 8, 1024


def _read_counters(d):
    """{dispatch id: {counter: value summed over its instances}} from a rocprofv3 --pmc CSV under directory d."""
    import csv
    import glob
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            dd = out.setdefault(int(r["Dispatch_Id"]), {})
            dd[r["Counter_Name"]] = dd.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def _read_durations(d):
    """{dispatch id: kernel duration in ns} from the rocprofv3 kernel trace under directory d."""
    import csv
    import glob
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            out[int(r["Dispatch_Id"])] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return out


def under_profiler() -> str:
    """Why this process looks profiled ('' when it does not): the rocprofiler tool library in LD_PRELOAD, or the
    ROCP_* / ROCPROF_* variables rocprofv3 sets for its child."""
    pre = os.environ.get("LD_PRELOAD", "")
    if "rocprof" in pre:
        return "LD_PRELOAD names a rocprofiler library"
    keys = sorted(k for k in os.environ if k.startswith(("ROCP_", "ROCPROF")))
    return f"{keys[0]} is set" if keys else ""


def collect_pmc(child_args, timeout_s=150):
    """HBM traffic, effective clock and MFMA-pipe occupancy of the dominant kernel, measured in this bench run: the
    same workload is launched by a child `bench.py --pmc-child` under rocprofv3, one counter pass per group of
    PMC_PASSES (FETCH_SIZE and WRITE_SIZE cannot share a pass: 3 + 2 TCC counters), with the kernel trace for the
    per-dispatch duration.  Corrections per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE reports half of the
    bytes of 16-B-per-lane reads on gfx950 (every weight load here is a 16-B buffer_load), so HBM bytes =
    2 x FETCH_SIZE + WRITE_SIZE (KiB); effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; MFMA pipe busy =
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).  Returns None when rocprofv3 is unavailable or a
    pass fails (the bench line then reports traffic null)."""
    import shutil
    import signal
    import statistics
    import tempfile
    why = under_profiler()
    if why:
        # rocprofv3 is a `#!/usr/bin/env python3` script: started from a process the profiler's tool library has
        # already attached to, it is an exec of a GPU-initialised process (refused on this pool)
        print(f"[bench] PMC passes skipped: this process runs under a profiler ({why})", file=sys.stderr, flush=True)
        return None
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    vals, durs = {}, {}
    with tempfile.TemporaryDirectory(prefix="ecnf_pmc_", dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        for k, counters in enumerate(PMC_PASSES):
            d = os.path.join(tmp, f"p{k}")
            cmd = [prof, "--pmc", *counters, "--kernel-trace", "--kernel-include-regex", "integrate_kernel",
                   "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child", *child_args]
            env = dict(os.environ, TMPDIR=tmp)
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, start_new_session=True)
            try:
                _, err = p.communicate(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                print(f"[bench] PMC pass {counters} timed out", file=sys.stderr, flush=True)
                return None
            if p.returncode != 0:
                print(f"[bench] PMC pass {counters} failed: {err.decode(errors='replace')[-800:]}", file=sys.stderr,
                      flush=True)
                return None
            for disp, cv in _read_counters(d).items():
                vals.setdefault(k, {})[disp] = cv
            if k == 0:
                durs = _read_durations(d)
    try:
        # the child runs one warm-up launch and then the measured ones: drop each pass's first dispatch
        def per_launch(k, name):
            ds = sorted(vals[k])[1:] or sorted(vals[k])
            return statistics.median(vals[k][x][name] for x in ds), ds
        fetch_kib, ds0 = per_launch(0, "FETCH_SIZE")
        write_kib, _ = per_launch(1, "WRITE_SIZE")
        gui, _ = per_launch(0, "GRBM_GUI_ACTIVE")
        busy, _ = per_launch(0, "SQ_VALU_MFMA_BUSY_CYCLES")
        dur_ns = statistics.median(durs[x] for x in ds0 if x in durs) if durs else None
    except (KeyError, ValueError, statistics.StatisticsError):
        return None
    clock = gui / N_XCD / (dur_ns * 1e-9) / 1e9 if dur_ns else None
    return {"hbm_bytes_per_launch": (2.0 * fetch_kib + write_kib) * 1024.0,
            "fetch_bytes_per_launch": 2.0 * fetch_kib * 1024.0, "write_bytes_per_launch": write_kib * 1024.0,
            "fetch_size_kib_raw": fetch_kib, "grbm_gui_active": gui, "sq_valu_mfma_busy_cycles": busy,
            "kernel_ms_in_pmc_run": dur_ns * 1e-6 if dur_ns else None, "clock_ghz_grbm": clock,
            "mfma_pipe_busy_frac": busy / (gui / N_XCD * N_SIMD) if gui else None,
            "source": "rocprofv3 --pmc (2 passes) + --kernel-trace of a child bench.py --pmc-child on the same "
                      "workload, inside this bench run; FETCH_SIZE doubled per the gfx950 16-B/lane correction"}


def cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline_child(cfg_name: str, n_mol: int, n_mol_1t: int, nfe: int, threads: int, repeats: int) -> dict:
    """(runs in a CPU-only child process, see cpu_baseline) the torch-CPU fp32 batched restatement (oracle/torch_ref.py,
    the batched-GEMM structure XLA builds from vmap) of the same Euler NFE-step sample (torch_ref.sample_euler's time
    grid) on `n_mol` molecules with `threads` threads and on `n_mol_1t` with one thread.  Every Euler step is timed
    on its own: the value is molecules / (NFE x the median step time) over the `repeats` x NFE steps, which a transient
    stall of the host (a slow first solve, another tenant) does not move; the whole-solve rate and the spread of the
    step times (10th-90th percentile / median) are reported beside it."""
    import numpy as np
    import torch
    from oracle import ecnf_oracle as O
    from oracle import torch_ref as R
    oc = O.CONFIGS[cfg_name]
    P = R.to_torch(O.init_params(oc, 0))
    rng = np.random.default_rng(0)
    z = rng.standard_normal((max(n_mol, n_mol_1t), oc.n_nodes * oc.dim)).astype(np.float32)
    x_all = torch.from_numpy(O.base_sample(z, oc))
    feat_all = torch.zeros((x_all.shape[0], oc.n_nodes), dtype=torch.int32)

    def solve(n, steps):
        x, feat, dt, tau, ts = x_all[:n].clone(), feat_all[:n], np.float32(1.0 / nfe), np.float32(0.0), []
        with torch.no_grad():
            while tau < 1.0 and len(ts) < steps:
                tn = np.float32(tau + dt)
                tn = np.float32(1.0) if tn > np.float32(1.0) - np.float32(1e-6) else tn
                t0 = time.perf_counter()
                v = R.vector_field(P, oc, x, torch.full((n,), float(tau), dtype=x.dtype), feat)
                x = x + float(np.float32(tn - tau)) * v
                ts.append(time.perf_counter() - t0)
                tau = tn
        return ts

    out = {}
    for key, th, n in (("all", threads, n_mol), ("one", 1, n_mol_1t)):
        torch.set_num_threads(th)
        solve(n, 5)                                              # warm-up at the timed batch shape
        steps = []
        for _ in range(repeats):
            steps += solve(n, nfe)
        med = float(np.median(steps))
        p10, p90 = np.percentile(steps, [10, 90])
        out[key] = {"median": n / (nfe * med), "whole_solve": n * repeats / sum(steps),
                    "spread": float((p90 - p10) / med), "seconds": sum(steps), "threads": torch.get_num_threads(),
                    "molecules": n, "steps_timed": len(steps)}
    return out


def cpu_baseline(cfg_name: str, n_mol: int, n_mol_1t: int, nfe: int, threads: int, repeats: int):
    """The CPU baseline, timed in a child process that never touches the GPU, with its OpenMP threads bound one per
    core of this process's affinity set (OMP_PROC_BIND=close, OMP_PLACES=cores, OMP_NUM_THREADS=threads) so the
    threads do not migrate; the median of `repeats` timed solves is the reported value and their spread is stated."""
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES="cores")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child",
           json.dumps([cfg_name, n_mol, n_mol_1t, nfe, threads, repeats])]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed: {r.stderr[-800:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start n rank processes of this script under torch.distributed.run as a CHILD (this process has not touched
    the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0,
                    help="GLOBAL molecules per step (default: 1024 at one rank, 65536 over several ranks)")
    ap.add_argument("--config", default="lj13")
    ap.add_argument("--nfe", type=int, default=100)
    ap.add_argument("--logprob", type=int, default=-1,
                    help="eval leg (sample + Hutchinson log-prob + target + ESS) passes (default 1)")
    ap.add_argument("--fp32-steps", type=int, default=2, help="launches of the strict-fp32 kernels timed (0 = skip)")
    ap.add_argument("--train-steps", type=int, default=10, help="timed training steps at N = 1 (0 = skip)")
    ap.add_argument("--train-batch", type=int, default=64, help="training batch (lj13.yaml: 64)")
    ap.add_argument("--ref-latency-samples", type=int, default=10,
                    help="calls of the reference's single-molecule QM9 sampling-time script (first = warm-up; 0 = skip)")
    ap.add_argument("--cpu-molecules", type=int, default=128, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-molecules-1t", type=int, default=24, help="bounded 1-thread CPU-baseline sample")
    ap.add_argument("--cpu-repeats", type=int, default=1, help="timed CPU-baseline solves (median step time reported)")
    ap.add_argument("--cpu-child", default="", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (multi-rank rehearsal)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--dump", default="", help="directory: each rank saves its shard's outputs (tests)")
    ap.add_argument("--pmc", type=int, default=-1,
                    help="measure HBM traffic / clock / MFMA busy with rocprofv3 counter passes of this workload "
                         "(default: on at one rank, off over several)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.cpu_child:   # the CPU baseline's child process (cpu_baseline): no GPU is touched
        print(json.dumps(cpu_baseline_child(*json.loads(args.cpu_child))), flush=True)
        return

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import numpy as np
    import torch
    import torch.distributed as dist
    from ecnf_amd import CONFIGS, init_params, param_count
    from ecnf_amd import _lib
    from ecnf_amd import distributed as D
    from ecnf_amd.engine import EcnfHandle, SolveOptions

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torch.distributed.run the process group forms at every world size (one rank included: the eval leg's
    # reductions then run through RCCL, tests/test_gpu_rccl.py); a plain `python bench.py` run has no group
    if "WORLD_SIZE" in os.environ:
        ndev = max(1, torch.cuda.device_count())
        local = local % ndev                  # one rank per GPU; folds ranks onto fewer GPUs only in rehearsals
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
        world = dist.get_world_size()         # the world the process group actually formed
        rank = dist.get_rank()
    dev = torch.device("cuda", local)
    cfg = CONFIGS[args.config]
    G = args.batch or (GLOBAL_BATCH_MULTI if world > 1 else 1024)
    lo, hi = D.shard_bounds(G, rank, world)
    B = hi - lo
    n_logprob = args.logprob if args.logprob >= 0 else 1

    h = EcnfHandle(cfg, init_params(cfg, 0), local)
    z = D.global_normal(G, cfg.event_dim, args.seed, lo, hi, dev)     # rows [lo, hi) of one global draw
    x0 = h.base_sample(z)
    feat = torch.zeros((B, cfg.n_nodes), device=dev, dtype=torch.int32)
    opts = SolveOptions(solver="euler", step_size=1.0 / args.nfe)

    def step():
        return h.integrate(x0, feat, 0.0, 1.0, opts, check_status=False)

    if args.pmc_child:
        # under rocprofv3 (collect_pmc): one warm-up launch, then the measured launches of the same workload
        for _ in range(1 + max(1, args.steps)):
            step()
        torch.cuda.synchronize(dev)
        return

    for _ in range(args.warmup):
        y1, _, nfe, _ = step()
    torch.cuda.synchronize(dev)
    nfe_seen = int(nfe.max()) if args.warmup and B else args.nfe

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        y1, _, nfe, status = step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    t_run = time.perf_counter() - t0
    barrier()
    t_max = max_over_ranks(t_run)
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if args.steps else 0.0
    assert int((status != 0).sum()) == 0 and torch.isfinite(y1).all()

    value = G * args.steps / t_max
    F = live_flops_per_eval(cfg)
    # algorithmic HBM bytes of one launch: x0 in, x1 / nfe / status out (fp32 / int32), one read of the weight set
    algo_bytes = B * (2 * cfg.event_dim * 4 + 8) + 4 * param_count(cfg)
    achieved = F * nfe_seen * B / (kernel_ms * 1e-3) / 1e12
    chain_mode = h.chain_arithmetic()
    peak = roofline_peak(cfg, chain_mode)
    Fx = executed_flops_per_eval(cfg, chain_mode)

    # the strict-fp32 kernels (every GEMM on v_mfma_f32_32x32x2_f32) on the same workload, for comparison
    fp32 = None
    if args.fp32_steps > 0 and B:
        h.set_precision("fp32")
        y1_32, _, _, _ = step()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.fp32_steps):
            y1_32, _, _, _ = step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        h.set_precision("split_f16")
        ms32 = e0.elapsed_time(e1) / args.fp32_steps
        fp32 = {"kernel_ms": ms32, "molecules_per_s_per_gpu": B / (ms32 * 1e-3),
                "achieved_tflops": F * nfe_seen * B / (ms32 * 1e-3) / 1e12,
                "max_abs_diff_vs_split": float((y1_32 - y1).abs().max())}

    # eval leg (setup_training.py:166-185): sample_and_log_prob_cnf(approx=True) -> target -> log_w -> ESS
    logprob = None
    if n_logprob > 0:
        from ecnf_amd import targets as T
        for i in range(n_logprob + 1):        # pass 0 warms up
            barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            ek0, ek1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ek0.record(stream)
            x1, dl, _, st = h.integrate(x0, feat, 0.0, 1.0, opts, divergence=_lib.DIV_HUTCHINSON, eps=z,
                                        check_status=False)
            ek1.record(stream)
            log_q = h.base_log_prob(x0) - dl          # sample_and_log_prob.py:147 (eps = z: the ref's quirk)
            log_p = T.lj_log_prob(x1, cfg.n_nodes, cfg.dim) if args.config == "lj13" else \
                T.dw_log_prob(x1, cfg.n_nodes, cfg.dim)
            log_w = log_p - log_q
            # reverse ESS of model samples (eval_batch_free_fn, setup_training.py:166-185); the forward ESS needs
            # samples of the TARGET (evaluation.py:10-22, on the test set: ecnf_amd.evaluation), not model samples
            _, rev = D.ess_from_device(log_w)         # one MAX + one SUM all-reduce (RCCL under nccl)
            mean_lq = D.masked_mean(log_q)
            torch.cuda.synchronize(dev)
            barrier()
            t_lp = max_over_ranks(time.perf_counter() - t1)
        # the backend that actually reduced the ESS / mean statistics: the formed process group's (RCCL for nccl),
        # or none in a plain one-process run (distributed._allreduce is then the identity)
        red = dist.get_backend() if dist.is_initialized() else None
        red = {"nccl": "RCCL", None: "local reductions (one process, no process group)"}.get(red, red)
        logprob = {"workload": f"{args.config} sample_and_log_prob_cnf (Hutchinson, Euler NFE={args.nfe}) + target "
                               f"log-density + ESS, {red}",
                   "reduced_by": red,
                   "molecules_per_s": G / t_lp, "ms": t_lp * 1e3,
                   # the divergence kernel alone (HIP events on its stream): primal + one tangent per evaluation
                   "kernel_ms": ek0.elapsed_time(ek1),
                   "achieved_tflops": 2 * F * nfe_seen * B / (ek0.elapsed_time(ek1) * 1e-3) / 1e12 if B else 0.0,
                   "tangent_kernels": h.chain_arithmetic(with_tangent=True), "rev_ess": float(rev),
                   "mean_log_q": float(mean_lq), "status_ok": bool(int((st != 0).sum()) == 0)}
        if args.dump:
            os.makedirs(args.dump, exist_ok=True)
            np.savez(os.path.join(args.dump, f"rank{rank}.npz"), lo=lo, hi=hi, z=z.cpu().numpy(),
                     x0=x0.cpu().numpy(), x1=y1.cpu().numpy(),
                     x1_lp=x1.cpu().numpy(), log_q=log_q.cpu().numpy(), log_w=log_w.cpu().numpy(),
                     rev_ess=float(rev), mean_log_q=float(mean_lq), world=world)

    # the reference's own timing script (examples/load_checkpoint_measure_sampling_time.py:101-119): qm9.yaml
    # network, ONE molecule per sample_cnf call with the default adaptive solve (Dopri5 + PIDController rtol = atol =
    # 1e-5), 10 calls of which the first is the warm-up; wall time per call incl. the host round trip.  Random-init
    # weights (the script loads a trained wandb checkpoint, unavailable offline), so the step count differs.
    ref_latency = None

    def ref_sampling_latency():
        qcfg = CONFIGS["qm9"]
        hq = EcnfHandle(qcfg, init_params(qcfg, 0), local)
        gq = torch.Generator(device=dev)
        gq.manual_seed(0)
        fq = torch.zeros((1, qcfg.n_nodes), device=dev, dtype=torch.int32)

        def calls(team_mode):
            # team_mode 0: the default (team mode: ecnf_team_workgroups(1) workgroups per molecule); 1: the batch path
            hq.set_team(team_mode)
            gq.manual_seed(0)
            times, nfes, xs = [], [], []
            for i in range(args.ref_latency_samples):
                zq = torch.randn((1, qcfg.event_dim), generator=gq, device=dev)
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                xq, _, nq, sq = hq.integrate(hq.base_sample(zq), fq, 0.0, 1.0, SolveOptions("dopri5", None))
                xs.append(xq.cpu())                    # the sample reaches the host, as jax's result does
                if i:
                    times.append(time.perf_counter() - t1)
                    nfes.append(int(nq.max()))
            hq.set_team(0)
            return times, nfes, xs

        G = hq.team_workgroups(1)
        times, nfes, xs = calls(0)
        times_b, _, xs_b = calls(1)
        del hq
        return {"workload": "qm9 sample_cnf, 1 molecule per call, Dopri5 + PID rtol=atol=1e-5 "
                            "(load_checkpoint_measure_sampling_time.py:101-119), random-init weights",
                "ms_median": 1e3 * float(np.median(times)), "ms_min": 1e3 * float(np.min(times)),
                "nfe_median": float(np.median(nfes)), "calls": len(times), "team_workgroups": G,
                "batch_path_ms_median": 1e3 * float(np.median(times_b)),
                "team_equals_batch_path": all(bool(torch.equal(a, b)) for a, b in zip(xs, xs_b))}

    if world == 1 and args.ref_latency_samples > 1:
        try:   # an auxiliary leg: its failure is reported in the line, never fails the headline measurement
            ref_latency = ref_sampling_latency()
        except Exception as e:  # noqa: BLE001
            ref_latency = {"error": f"{type(e).__name__}: {e}"}

    # training leg (SURVEY 8f rank 3, lj13.yaml training: Adam, batch 64): one flow_matching_update_fn step =
    # loss + reverse-mode gradient + Adam, on the same device (N = 1 only)
    train = None
    if world == 1 and args.train_steps > 0:
        from ecnf_amd import train as TRN
        tr = TRN.Trainer(cfg, max_batch=args.train_batch, device=local)
        p = tr.device_params(init_params(cfg, 0))
        mu, nu = torch.zeros_like(p), torch.zeros_like(p)
        gtr = torch.Generator(device=dev)
        gtr.manual_seed(5)
        xd = h.base_sample(torch.randn((args.train_batch, cfg.event_dim), generator=gtr, device=dev))
        xb = h.base_sample(torch.randn((args.train_batch, cfg.event_dim), generator=gtr, device=dev))
        tt = torch.rand((args.train_batch,), generator=gtr, device=dev)
        ft = torch.zeros((args.train_batch, cfg.n_nodes), device=dev, dtype=torch.int32)
        for i in range(args.train_steps + 2):
            if i == 2:
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            loss, grad = tr.loss_and_grad(p, xd, xb, tt, ft)
            tr.adam_update(grad, p, mu, nu, None, lr=1e-4, count=i + 1)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / args.train_steps
        train = {"workload": f"{args.config} flow-matching training step (loss + reverse-mode gradient + Adam), "
                             f"batch {args.train_batch}, strict-fp32 MFMA GEMMs",
                 "ms_per_step": ms, "steps_per_s": 1e3 / ms, "molecules_per_s": args.train_batch * 1e3 / ms,
                 "loss": float(loss)}

    # HBM traffic, effective clock and MFMA occupancy of this workload's kernel, from counter passes run now
    pmc = None
    if rank == 0 and (args.pmc > 0 or (args.pmc < 0 and world == 1)):
        pmc = collect_pmc(["--config", args.config, "--batch", str(G), "--nfe", str(args.nfe), "--seed",
                           str(args.seed), "--steps", "2"])

    cpu = None
    if rank == 0 and world == 1 and args.cpu_molecules > 0:
        threads = args.cpu_threads or len(os.sched_getaffinity(0))
        cb = cpu_baseline(args.config, args.cpu_molecules, args.cpu_molecules_1t, args.nfe, threads,
                          max(1, args.cpu_repeats))
        a1, o1 = cb["all"], cb["one"]
        cpu = {"value": a1["median"], "unit": "molecules/s", "cores": a1["threads"], "kind": "port",
               "whole_solve_value": a1["whole_solve"], "step_time_spread_p10_p90": a1["spread"],
               "value_1_thread": o1["median"], "whole_solve_value_1_thread": o1["whole_solve"],
               "cpu_model": cpu_model(),
               "sample": f"{args.cpu_molecules} {args.config} molecules x {args.nfe} Euler steps "
                         f"(x{max(1, args.cpu_repeats)}) on {a1['threads']} threads bound to the affinity set's cores "
                         f"({a1['seconds']:.1f} s) and {args.cpu_molecules_1t} on 1 thread ({o1['seconds']:.1f} s); "
                         f"value = molecules / (NFE x median step time); torch-CPU fp32 batched restatement "
                         f"(oracle/torch_ref.py) in a CPU-only child process"}

    if rank == 0:
        out = {
            "metric": "sampled molecules/sec (fixed-step ODE, NFE=100), LJ13 N=13",
            "value": value,
            "unit": "molecules/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3 if args.steps else 0.0,
            "higher_is_better": True,
            "scaling": "strong" if world > 1 and not args.batch else "weak",
            "vs_baseline": None,
            "dtype": "f32 (split_f16x3: fp32 operands as two fp16 pieces, 3 cross terms, fp32 accumulate)"
                     if chain_mode == "split_f16" else "f32",
            "data": "synthetic (seeded zero-CoM Gaussian x0, flax-default random-init lj13 weights)",
            "config": {"workload": f"{args.config} sample, Euler NFE={nfe_seen}, global batch {G} "
                                   f"({B} per GPU on rank 0)",
                       "n_nodes": cfg.n_nodes, "batch_per_gpu": B, "global_batch": G,
                       "nfe": nfe_seen, "solver": "euler", "parallelism": f"dp{world}",
                       "dist_backend": dist.get_backend() if dist.is_initialized() else None},
            "matmul": {"gemms": chain_mode, "tangent_kernels": h.chain_arithmetic(True) + " edge chains",
                       "accumulate": "f32", "strict_fp32": fp32},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak,
                         "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                         "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE, this run)",
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "kernel": "integrate_kernel", "kernel_ms": kernel_ms,
                         "flop_per_launch": F * nfe_seen * B,
                         "flop_basis": "live dense-contraction FLOPs per EGNN eval (SURVEY 8d F minus the last "
                                       "block's dead h update) x NFE x batch",
                         # the FLOPs the kernel executes (block-1 pair tiles skip the mirrored half of block 1's edge
                         # work) and the fraction of the same ceiling they reach
                         "flop_executed_per_launch": Fx * nfe_seen * B,
                         "frac_executed": achieved * (Fx / F) / peak,
                         "frac_vs_fp32_mfma_peak": achieved / PEAK_FP32_MFMA_TFLOPS,
                         "pmc": pmc,
                         "frac_at_grbm_clock": (achieved / (peak * pmc["clock_ghz_grbm"] / 2.4)
                                                if pmc and pmc.get("clock_ghz_grbm") else None),
                         "peak_basis": (f"GEMM FLOPs at the dense 16-bit MFMA peak / {SPLIT_TERMS[chain_mode]} split "
                                        "terms, vector FLOPs at the fp32 peak") if chain_mode in SPLIT_TERMS
                                       else "fp32 MFMA peak"},
            "logprob": logprob,
            "train": train,
            "ref_sampling_latency": ref_latency,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
