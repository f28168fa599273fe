"""PinSAGE train-step throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4] [--scaling weak|strong]
                    [--no-cpu-baseline]

A step = sample_batch (reference RNG semantics, host) + PinSage.train_batch
(fused HIP forward of the query/positive/negative ids, loss, backward, Adam)
on a synthetic playlist graph resident in HBM.  N > 1: one process per GPU
(torch.distributed over RCCL), each rank trains batch_size triples per step
(weak scaling), gradients all-reduced.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gcn-song-embeddings_amd"))
sys.path.insert(0, REPO)

CONFIGS = {
    # BASELINE.json configs[1]: dataset_final_intersect-like, 2-layer, fanout 10, batch 512
    "c2": dict(workload="synthetic dataset_final_intersect-scale playlist graph, 2-layer PinSAGE, "
                        "fanout 10, batch 512", n_tracks=100_000, n_cols=25_000,
               memberships=1_000_000, d_in=512, n_layers=2, T=10, batch=512),
    "c3": dict(workload="synthetic dataset_large-scale playlist graph, 2-layer PinSAGE, fanout 25, "
                        "batch 2048", n_tracks=1_000_000, n_cols=250_000, memberships=10_000_000,
               d_in=512, n_layers=2, T=25, batch=2048),
    # memberships are drawn with repeats and deduplicated: 53.6M draws leave 50.0M distinct
    # track-collection pairs = 100.0M directed edges (tests/test_gpu_configs.py checks it)
    "c4": dict(workload="synthetic 10M nodes / 100M edges, 128-d features, 2-layer, per-GPU batch 512",
               n_tracks=8_000_000, n_cols=2_000_000, memberships=53_600_000, d_in=128, n_layers=2,
               T=10, batch=512, global_batch=4096),
    # BASELINE.json configs[4]: 100M nodes / 1B edges, d 256, 3 layers, fanout 50. Built
    # on the device (a host build takes ~10 min); the [n, 100] host table would be 128 GB,
    # so the model's T=50 table is made and kept in HBM (precompute_device_table); one
    # 512-triple step reaches ~10^6 layer-0 nodes, so it runs in slices of `micro_batch`
    # triples with recompute (PinSage.micro_batch)
    "c5": dict(workload="synthetic 100M nodes / 1B edges, 256-d features, 3-layer fanout 50, "
                        "per-GPU batch 512 in micro-batches of 16 triples", n_tracks=80_000_000,
               n_cols=20_000_000, memberships=536_000_000, d_in=256, n_layers=3, T=50, batch=512,
               global_batch=4096, micro_batch=16, device_build=True),
}
# --scaling strong: the global batch stays fixed (C4 B_global 4096, per-GPU
# 4096/g); configs without a global_batch keep their batch as the global one

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E peak
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)
SPLIT_BF16_CEIL_TFLOPS = PEAK_BF16_TFLOPS / 6  # fp32 products at six bf16 MFMAs each


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def setup_dist(n_gpus):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # PINSAGE_DIST_BACKEND=gloo rehearses the data-parallel path with ranks
        # sharing one GPU (device = local rank mod the visible GPUs); the
        # multi-GPU run uses nccl (= RCCL over xGMI)
        backend = os.environ.get("PINSAGE_DIST_BACKEND", "nccl")
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            torch.distributed.init_process_group(backend)
    return rank, world


def build_problem_device(cfg, seed=0):
    """C5-sized inputs drawn on the device (synthetic.make_playlist_graph_device):
    graph, N(0,1) features z-scored per column, positives (host, for the sampler)."""
    import graph
    import synthetic
    t0 = time.time()
    dev = torch.device("cuda")
    log(f"[bench] building synthetic graph on the device: {cfg['n_tracks']} tracks, "
        f"{cfg['n_cols']} collections, {cfg['memberships']} memberships")
    indptr, indices = synthetic.make_playlist_graph_device(cfg["n_tracks"], cfg["n_cols"], cfg["memberships"],
                                                           seed=seed, device=dev)
    g = graph.DeviceCSRGraph(indptr, indices)
    log(f"[bench]   CSR built ({time.time()-t0:.1f}s): n_all={g.number_of_nodes()} edges={int(indices.shape[0])}")
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + 1)
    feats = torch.empty((cfg["n_tracks"], cfg["d_in"]), dtype=torch.float32, device=dev)
    for i in range(0, cfg["n_tracks"], 1 << 22):
        feats[i:i + (1 << 22)].normal_(generator=gen)
    # z-scored per column (spotify_graph.py:77-79) in row chunks: no full-size temporaries
    ch = 1 << 20
    n = cfg["n_tracks"]
    mean = sum(feats[i:i + ch].sum(0, dtype=torch.float64) for i in range(0, n, ch)) / n
    var = sum(((feats[i:i + ch].double() - mean) ** 2).sum(0) for i in range(0, n, ch)) / (n - 1)
    std = var.sqrt() + 1e-12
    for i in range(0, n, ch):
        feats[i:i + ch] = ((feats[i:i + ch].double() - mean) / std).float()
    pos = synthetic.make_positives_device(indptr, indices, cfg["n_tracks"], 5 * cfg["n_tracks"], seed=seed + 2)
    log(f"[bench] features and {pos.shape[0]} positives in {time.time()-t0:.1f}s")

    class _PG:
        n_all = g.number_of_nodes()
        n_edges = int(indices.shape[0])
    return _PG(), g, feats, pos


def build_problem(cfg, seed=0):
    import graph
    import synthetic
    if cfg.get("device_build"):
        return build_problem_device(cfg, seed)
    t0 = time.time()
    log(f"[bench] building synthetic graph: {cfg['n_tracks']} tracks, {cfg['n_cols']} collections, "
        f"{cfg['memberships']} memberships")
    pg = synthetic.make_playlist_graph(cfg["n_tracks"], cfg["n_cols"], cfg["memberships"], seed=seed)
    log(f"[bench]   memberships drawn in {time.time()-t0:.1f}s")
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices)
    log(f"[bench]   CSR built ({time.time()-t0:.1f}s)")
    rng = np.random.default_rng(seed + 1)
    feats = torch.from_numpy(rng.standard_normal((cfg["n_tracks"], cfg["d_in"]), dtype=np.float32))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * cfg["n_tracks"], seed=seed + 2,
                                                    csr=(indptr, indices)))
    log(f"[bench] graph n_all={pg.n_all} edges={pg.n_edges} built in {time.time()-t0:.1f}s")
    return pg, g, feats, pos


def precompute(g, cfg, mode):
    import pinsage_model as pm
    pm.set_rng_mode(mode)
    torch.manual_seed(0)
    torch.cuda.synchronize()
    t0 = time.time()
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):  # progress prints must not reach the JSON line
        if cfg.get("device_build"):  # the model's T columns of the top-100, kept in HBM
            nb = pm.precompute_device_table(g, cfg["n_tracks"], pm.DEF_HOPS, pm.DEF_ALPHA, cfg["T"],
                                            pm.DEF_T_PRECOMP)
        else:
            nb = pm.precompute_neighborhoods_topt(g, cfg["n_tracks"], pm.DEF_HOPS, pm.DEF_ALPHA,
                                                  pm.DEF_T_PRECOMP, None)
    torch.cuda.synchronize()
    dt = time.time() - t0
    pm.set_rng_mode("mt19937")
    return nb, dt


def kernel_table(engine):
    import ctypes
    import _native as nat
    L = nat.lib()
    L.pinsage_engine_timing_collect(engine.h)
    out = {}
    i = 0
    name = ctypes.create_string_buffer(128)
    ms = ctypes.c_double()
    calls = ctypes.c_int64()
    while L.pinsage_engine_timing_get(engine.h, i, name, 128, ctypes.byref(ms), ctypes.byref(calls)) == 0:
        out[name.value.decode()] = (ms.value, calls.value)
        i += 1
    return out


def pmc_traffic(config, site):
    """HBM bytes per launch of `site` from the newest committed rocprofv3 --pmc
    summary (profiles/rNN/pmc_<config>_*.json, written by the PMC passes that
    tools/pmc_summary.py documents); None when there is none for this config."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"pmc_{config}_*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("site") == site and d.get("config") == config:
            return d["hbm_bytes_per_launch"], os.path.relpath(path, REPO), d.get("mfma_busy")
    return None, None, None


def host_cores():
    """(threads to use, facts): the host's physical cores (lscpu), capped by what
    this process may run on (affinity, cgroup CPU quota -- a GPU box grants one
    job a share of a large host)."""
    import subprocess
    facts = {}
    try:
        out = subprocess.run(["lscpu", "-p=Core,Socket"], capture_output=True, text=True, timeout=10).stdout
        facts["physical_cores"] = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")})
    except Exception:
        pass
    facts["affinity_cpus"] = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            facts["cgroup_cpu_quota"] = int(q) / int(per)
    except Exception:
        pass
    cands = [facts.get("physical_cores"), facts["affinity_cpus"], facts.get("cgroup_cpu_quota")]
    threads = max(1, int(min(c for c in cands if c)))
    return threads, facts


def cpu_baseline(cfg, pg, feats, pos, nbhds, seconds=45.0, steps=20, warmup=3):
    """The oracle's restatement of the reference train step (dense clone
    put_embeddings, f64 aggregation, torch CPU) on the same workload, on all the
    physical cores this job may use: `warmup` untimed steps,
    then the median of `steps` timed ones (fewer only if `seconds` runs out)."""
    from oracle import oracle as orc
    import pinsage_model as pm
    threads, facts = host_cores()
    torch.set_num_threads(threads)
    # the restatement's backward at the reference init makes denormals the reference's op
    # order does not (its step time grew 1.6 -> 8 s); flushed so it times the algorithm
    # (tools/refcpu_ratio.py: refcpu / reference time ratio with the same setting)
    torch.set_flush_denormal(True)
    torch.manual_seed(1)
    dims = (cfg["d_in"], 512, 128)
    tmp = {}
    in_dims = [dims[0]] + [dims[2]] * (cfg["n_layers"] - 1)
    for i in range(cfg["n_layers"]):
        c = pm.ConvLayer(in_dims[i], dims[2], dims[1])  # CPU params, reference init
        for k, v in c.state_dict().items():
            tmp[f"conv_layers.{i}.{k}"] = v.numpy()
    G1 = torch.nn.Linear(128, 128)
    G2 = torch.nn.Linear(128, 128, bias=False)
    tmp.update({"G1.weight": G1.weight.detach().numpy(), "G1.bias": G1.bias.detach().numpy(),
                "G2.weight": G2.weight.detach().numpy()})
    tr = orc.RefTrainer(tmp, feats, nbhds[0].numpy(), nbhds[1].numpy(), n_layers=cfg["n_layers"],
                        T=cfg["T"])
    mt = orc.MT(2)
    for _ in range(warmup):
        b, _ = orc.sample_batch_easy(mt, pos.numpy(), cfg["n_tracks"], cfg["batch"])
        tr.step(b)
    times = []
    t_start = time.time()
    while len(times) < steps and (time.time() - t_start) < seconds:
        t0 = time.time()
        b, _ = orc.sample_batch_easy(mt, pos.numpy(), cfg["n_tracks"], cfg["batch"])
        tr.step(b)
        times.append(time.time() - t0)
    t_step = float(np.median(times))
    torch.set_flush_denormal(False)
    # refcpu / reference time ratio, measured in the dev container (the only place the
    # reference runs) at the threads it has (8) and 4, tools/refcpu_ratio.py
    ratio, ratio_t4 = None, None
    rp = os.path.join(REPO, "profiles", "r06", "refcpu_ratio_t8.json")
    if os.path.isfile(rp):
        ratio = json.load(open(rp)).get("refcpu_over_reference")
    rp4 = os.path.join(REPO, "profiles", "r06", "refcpu_ratio_t4.json")
    if os.path.isfile(rp4):
        ratio_t4 = json.load(open(rp4)).get("refcpu_over_reference")
    return dict(value=3 * cfg["batch"] / t_step, unit="target nodes/s", cores=threads, kind="port",
                sample=f"median of {len(times)} timed train steps after {warmup} untimed ones, of the "
                       f"oracle's reference restatement (torch CPU, {threads} threads) on the same synthetic "
                       f"graph and config",
                flush_denormal=True,
                flush_denormal_note="torch.set_flush_denormal(True) while timing: the restatement's backward "
                                    "at the reference init produces denormals the reference's op order does "
                                    "not (1.6 -> 8 s per step without the flush); refcpu_over_reference was "
                                    "measured with the same setting",
                ms_per_step=t_step * 1e3, host=facts, refcpu_over_reference=ratio,
                refcpu_over_reference_t4=ratio_t4,
                refcpu_over_reference_source="profiles/r06/refcpu_ratio_t8.json / _t4.json (dev container, "
                                             "8 / 4 threads: the container has 8 CPUs, so the 16-thread ratio "
                                             "cannot be measured where the reference runs; < 1 means the "
                                             "restatement timed here is FASTER than the reference, i.e. the "
                                             "reported baseline is conservative)")


def launch_ranks(n_gpus):
    """`bench.py --gpus N` (N > 1) started without a launcher: run the same
    command under torch.distributed.run, one rank per GPU, as a child process
    (nothing here has touched the GPU, so no exec is involved), relay its
    output and exit with its code.  Started BY a launcher, WORLD_SIZE must
    equal --gpus."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != n_gpus:
            raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world} (launch one rank per GPU)")
        return
    if n_gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n_gpus} without a launcher: {' '.join(cmd)}")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    raise SystemExit(subprocess.call(cmd, env=env))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 50 (c5: 3)")
    ap.add_argument("--warmup", type=int, default=None, help="default 5 (c5: 1)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--scale", type=float, default=1.0,
                    help="rehearsal only: scale the graph (tracks, collections, memberships)")
    ap.add_argument("--precompute-rng", default="philox", choices=["philox", "mt19937"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: per-GPU batch fixed; strong: global batch fixed (per-GPU = global / N)")
    ap.add_argument("--sampling", default="table", choices=["table", "fly"],
                    help="table: the precomputed top-T neighbourhoods (the reference's default path); "
                         "fly: every call walks its nodes' neighbourhoods inside the step "
                         "(relevant_nodes_per_layer, pinsage_model.py:142-154), RNG per --precompute-rng")
    args = ap.parse_args()
    launch_ranks(args.gpus)
    cfg = dict(CONFIGS[args.config])
    if args.scale != 1.0:
        for k in ("n_tracks", "n_cols", "memberships"):
            cfg[k] = max(1000, int(cfg[k] * args.scale))
        cfg["workload"] += f" [REHEARSAL: graph scaled by {args.scale}]"
    micro = cfg.get("micro_batch")
    if args.steps is None:
        args.steps = 3 if micro else 50
    if args.warmup is None:
        args.warmup = 1 if micro else 5
    rank, world = setup_dist(args.gpus)
    if args.scaling == "strong":
        gb = cfg.get("global_batch", cfg["batch"])
        if gb % world:
            raise SystemExit(f"--scaling strong: global batch {gb} not divisible by {world} ranks")
        cfg["batch"] = gb // world

    import pinsage_training as pt
    import _native as nat
    nat.require_gpu()
    pg, g, feats, pos = build_problem(cfg)
    nbhds, t_pre = precompute(g, cfg, args.precompute_rng)
    hops = cfg["n_tracks"] * 500
    log(f"[bench] precompute ({args.precompute_rng}) {t_pre:.2f}s = {hops/t_pre/1e6:.1f} M hops/s")
    t_pre_warm = None
    if t_pre < 2.0 and not micro:  # the first call pays one-time costs (code objects, CSR upload): time it again
        _, t_pre_warm = precompute(g, cfg, args.precompute_rng)
        log(f"[bench] precompute again (warm) {t_pre_warm * 1e3:.1f} ms")

    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        g.nbhds_path = os.path.join(tmp, "nb.pt")
        if not cfg.get("device_build"):
            torch.save(nbhds, g.nbhds_path)
        torch.manual_seed(0)
        tr = pt.PinSage(g, cfg["n_tracks"], feats.cuda(), pos, log=False, load_save=False,
                        nbhds=nbhds if cfg.get("device_build") else None)
        # BASELINE config: n_layers / fanout / batch (bound before the model, as the reference does)
        if tr.T != cfg["T"] or tr.n_layers != cfg["n_layers"]:
            import pinsage_model as pm
            tr.T, tr.n_layers = cfg["T"], cfg["n_layers"]
            torch.manual_seed(0)
            tr.model = pm.PinSageModel(g, tr.n, tr.n_layers, tr.dimensions, tr.n_hops, tr.alpha, tr.T, tr.nbhds)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.scheduler = torch.optim.lr_scheduler.ExponentialLR(tr.optimizer, tr.decay)
        if args.sampling == "fly":
            import pinsage_model as pm
            pm.set_rng_mode(args.precompute_rng)
            torch.manual_seed(0)
            tr.model = pm.PinSageModel(g, tr.n, tr.n_layers, tr.dimensions, tr.n_hops, tr.alpha, tr.T, None)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.scheduler = torch.optim.lr_scheduler.ExponentialLR(tr.optimizer, tr.decay)
            cfg["workload"] += " [sampling on the fly: walks + top-T per layer inside every step]"
        tr.batch_size = cfg["batch"]
        tr.micro_batch = micro
        torch.manual_seed(1234)  # same global batches on every rank

        def step():
            batch, _ = tr.next_batch()
            return tr.train_batch(batch)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t_sample = t_enqueue = 0.0
        fz = tr._fused
        w0 = fz.ring_wait_s() if fz is not None else 0.0
        st0 = fz.stepper_stats() if fz is not None and fz.stepper is not None else None
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ta = time.perf_counter()
            batch, _ = tr.next_batch()
            tb = time.perf_counter()
            loss = tr.train_batch(batch)[0]
            t_sample += tb - ta
            t_enqueue += time.perf_counter() - tb
        t_wait = (fz.ring_wait_s() - w0) if fz is not None else 0.0
        native_step = bool(fz is not None and fz.stepper is not None)
        st_stats = fz.stepper_stats() if native_step else None
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t1 = time.perf_counter()
        elapsed = t1 - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            elapsed = float(t.item())
        ms_per_step = elapsed / args.steps * 1e3
        if pt._HOST_T is not None:
            log("[bench] host ms/step by section: " +
                json.dumps({k: round(v / (args.steps + args.warmup) * 1e3, 4) for k, v in pt._HOST_T.items()}))
        value = 3 * cfg["batch"] * world * args.steps / elapsed

        gemm_choices = tr._fused.tuned_choices if tr._fused is not None else None
        # per-kernel timing pass (HIP events on the launch stream), separate from the timed
        # loop; runs the same kernels eagerly (events are not recorded inside the graph)
        fused_any = tr._fused if tr._fused is not None else getattr(tr, "_fused_fly", None)
        if fused_any is not None:
            fused_any.use_graph = False
        eng = tr.model.runner().engine
        nat.lib().pinsage_engine_timing(eng.h, 1)
        n_t = 1 if micro else max(5, min(20, args.steps))
        sizes = []
        hold_stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(n_t):
            # hold the stream while the host queues the step, so the events time the
            # kernels back to back (an eager step's host enqueue is ~0.5 ms: without
            # the hold, an idle GPU would charge each launch's host gap to its kernel)
            if not micro:
                nat.lib().pinsage_stream_hold(3000, hold_stream)
            step()
            torch.cuda.synchronize()
            off = eng.off
            # micro-batched: the frontier of the last slice's outputs-only forward
            rn = tr.model.runner()
            ws = fused_any.ws if fused_any is not None else (rn._ws if rn._ws is not None else rn.last_ws)
            cN0 = int(eng.view(ws, int(off.count_N[0]), torch.int32, 1).item())
            cS0 = int(eng.view(ws, int(off.count_S[0]), torch.int32, 1).item())
            cN1 = (int(eng.view(ws, int(off.count_N[1]), torch.int32, 1).item())
                   if cfg["n_layers"] > 1 else 0)
            sizes.append((cN0, cS0, cN1))
        kt = kernel_table(eng)
        nat.lib().pinsage_engine_timing(eng.h, 0)
        os.chdir(cwd)

    U0 = float(np.mean([s[0] for s in sizes]))
    F0 = float(np.mean([s[1] for s in sizes]))
    U1 = float(np.mean([s[2] for s in sizes]))
    d, hid, T = cfg["d_in"], 512, cfg["T"]
    q_ms, q_calls = kt.get("fwd.q_gemm.l0", (0.0, 1))
    q_avg = q_ms / max(q_calls, 1)
    q_flops = 2.0 * U0 * d * hid
    achieved_tf = q_flops / (q_avg * 1e-3) / 1e12 if q_avg > 0 else 0.0
    # the gather kernel: the fused aggregation + W projection (fwd.aggw.l0), or the
    # aggregation alone when the engine runs them as two launches (PINSAGE_FUSED_AGGW=0)
    fused = "fwd.aggw.l0" in kt
    a_site = "fwd.aggw.l0" if fused else "fwd.agg.l0"
    a_ms, a_calls = kt.get(a_site, (0.0, 1))
    a_avg = a_ms / max(a_calls, 1)
    # the aggregation reads each of the U0 distinct q rows from HBM at most once (repeats
    # of a popular row are L2/Infinity-Cache hits): unique bytes are the HBM bound;
    # logical bytes (every slot's row) are reported as the cache-served gather rate
    agg_bytes = U0 * hid * 4 + F0 * T * 8 + F0 * hid * 4
    agg_logical = F0 * T * hid * 4 + F0 * T * 8 + F0 * hid * 4
    agg_flops = 0.0
    if fused:
        # + the gathered self rows, W, and the outputs y and row norms (agg is still
        # written: the W weight gradient reads it)
        extra = F0 * d * 4 + (d + hid) * 128 * 4 + F0 * 128 * 4 + F0 * 4
        agg_bytes += extra
        agg_logical += extra
        agg_flops = 2.0 * F0 * (d + hid) * 128
    # layer 1's Q projection fused into this kernel (engine.hip next_q: no
    # fwd.q_gemm.l1 launch): every output row's product with Q1 (hid x 128) is
    # computed, the U1 rows of layer 1's neighbour set are stored
    next_q = fused and cfg["n_layers"] > 1 and "fwd.q_gemm.l1" not in kt
    if next_q:
        agg_flops += 2.0 * F0 * 128 * hid
        nq_bytes = hid * 128 * 4 + hid * 4 + U1 * hid * 4
        agg_bytes += nq_bytes
        agg_logical += nq_bytes
    # committed PMC summaries are keyed by config (+ the per-GPU batch when it is not the
    # config's own, e.g. c4_b4096 = C4's global batch on one GPU)
    pmc_key = args.config if cfg["batch"] == CONFIGS[args.config]["batch"] else f"{args.config}_b{cfg['batch']}"
    a_traffic, a_traffic_src, _ = pmc_traffic(pmc_key, a_site)
    kernels = {k: {"avg_ms": v[0] / max(v[1], 1), "calls": v[1]} for k, v in sorted(kt.items())}
    traffic, traffic_src, mfma_busy = pmc_traffic(pmc_key, "fwd.q_gemm.l0")
    prec = nat.lib().pinsage_gemm_get_prec()
    gemm_arith = ("split bf16: each fp32 operand = hi + mid + lo bf16 (exact to 2^-26), six "
                  "v_mfma_f32_32x32x16_bf16 products per 16-k step, fp32 accumulation; achieved/peak are "
                  "algorithmic fp32 FLOP against the fp32 MFMA peak, executed bf16 MFMA work is 6x "
                  "(mfma_busy_pmc counts those cycles)" if prec == 1 else
                  "v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains)")
    q_roof = {"bound": "mfma", "kernel": "fwd.q_gemm.l0 (gather + Q projection on MFMA)",
              "arithmetic": gemm_arith,
              "achieved": achieved_tf, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
              "frac": achieved_tf / PEAK_FP32_TFLOPS, "traffic": traffic,
              # the ceiling of the arithmetic it runs: six bf16 MFMAs per fp32 product
              "split_bf16_ceiling": SPLIT_BF16_CEIL_TFLOPS,
              "frac_split_bf16_ceiling": achieved_tf / SPLIT_BF16_CEIL_TFLOPS,
              "traffic_source": traffic_src, "mfma_busy_pmc": mfma_busy,
              "algorithmic_per_launch": q_flops, "avg_launch_ms": q_avg,
              "algorithmic_bytes_per_launch": 4.0 * (U0 * d + d * hid + U0 * hid)}
    # the layer-0 Q weight gradient (dQ0 = dpq^T h[q_src], dQb, Adam on Q0: the
    # step's last launch), the same 2 U0 d hid FLOP
    w_ms, w_calls = kt.get("bwd.q_wgrad.l0", (0.0, 1))
    w_avg = w_ms / max(w_calls, 1)
    w_tf = q_flops / (w_avg * 1e-3) / 1e12 if w_avg > 0 else 0.0
    w_traffic, w_traffic_src, w_busy = pmc_traffic(pmc_key, "bwd.q_wgrad.l0")
    w_roof = {"bound": "mfma", "kernel": "bwd.q_wgrad.l0 (dQ0 = dpq^T h[q_src] + bias sums + Q0's Adam step)",
              "arithmetic": gemm_arith, "achieved": w_tf, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
              "frac": w_tf / PEAK_FP32_TFLOPS, "traffic": w_traffic,
              "split_bf16_ceiling": SPLIT_BF16_CEIL_TFLOPS,
              "frac_split_bf16_ceiling": w_tf / SPLIT_BF16_CEIL_TFLOPS,
              "traffic_source": w_traffic_src, "mfma_busy_pmc": w_busy,
              "algorithmic_per_launch": q_flops, "avg_launch_ms": w_avg,
              # dpq rows + gathered h rows + dQ0 written + Q0's p / m / v read and written
              "algorithmic_bytes_per_launch": 4.0 * (U0 * hid + U0 * d + 7 * d * hid + 4 * hid)}
    # `roofline` is the dominant (longest) of the two launches; the other beside it
    roof, roof_other = (w_roof, q_roof) if w_avg > q_avg else (q_roof, w_roof)
    result = {
        "metric": "PinSAGE train-step nodes/sec (2-hop, batch 512) at 1/2/4/8 MI355X",
        "value": value,
        "unit": "target nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded playlist graph, N(0,1) features, co-membership positives)",
        "config": {"workload": cfg["workload"], "n_tracks": cfg["n_tracks"], "n_cols": cfg["n_cols"],
                   "memberships": cfg["memberships"], "d_in": cfg["d_in"], "hidden": hid, "out": 128,
                   "n_layers": cfg["n_layers"], "fanout": T, "batch_per_gpu": cfg["batch"],
                   "global_batch": cfg["batch"] * world, "parallelism": f"dp{world}",
                   "batch_rng": "mt19937 (reference-exact)", "sampling": args.sampling},
        "roofline": roof,
        "roofline_other": roof_other,
        "gather_kernel": {"kernel": a_site + (" (weighted aggregation + [h_self || agg] W projection, "
                                              "bias, lrelu, row L2 norm in one launch"
                                              + (", + layer 1's Q projection of its rows" if next_q else "")
                                              + ")" if fused else ""),
                          "fused_next_q": next_q,
                          "bound": "hbm", "avg_launch_ms": a_avg,
                          "achieved_GBs": agg_bytes / (a_avg * 1e-3) / 1e9 if a_avg > 0 else 0.0,
                          "peak_GBs": PEAK_HBM_GBS, "frac": (agg_bytes / (a_avg * 1e-3) / 1e9 / PEAK_HBM_GBS
                                                             if a_avg > 0 else 0.0),
                          "algorithmic_bytes": agg_bytes,
                          "traffic": a_traffic, "traffic_source": a_traffic_src,
                          "logical_bytes": agg_logical,
                          "logical_GBs": agg_logical / (a_avg * 1e-3) / 1e9 if a_avg > 0 else 0.0,
                          "mfma_flops": agg_flops,
                          "mfma_frac": (agg_flops / (a_avg * 1e-3) / 1e12 / PEAK_FP32_TFLOPS
                                        if a_avg > 0 else 0.0),
                          # floors: algorithmic bytes at HBM peak, its projection at the fp32 MFMA
                          # peak; "frac_of_floor" = the larger floor (perfect overlap) / measured
                          "floor_hbm_ms": agg_bytes / PEAK_HBM_GBS / 1e6,
                          "floor_mfma_ms": agg_flops / PEAK_FP32_TFLOPS / 1e9,
                          "frac_of_floor": (max(agg_bytes / PEAK_HBM_GBS / 1e6, agg_flops / PEAK_FP32_TFLOPS / 1e9)
                                            / a_avg if a_avg > 0 else 0.0),
                          "frac_of_serial_floor": ((agg_bytes / PEAK_HBM_GBS / 1e6 + agg_flops / PEAK_FP32_TFLOPS / 1e9)
                                                   / a_avg if a_avg > 0 else 0.0),
                          "note": "algorithmic = unique q rows + index/weight + agg"
                                  + (" + self rows + W + y/norm outputs" if fused else "")
                                  + (" + Q1 weights and the U1 q rows it stores (flops: every row x Q1)"
                                     if next_q else "")
                                  + "; logical counts every (row, slot) read, most served by L2 / "
                                    "Infinity Cache"},
        "frontier": {"U0_mean": U0, "F0_mean": F0, "U1_mean": U1},
        "host_ms_per_step": {"sample_batch": t_sample / args.steps * 1e3,
                             "train_batch_enqueue": t_enqueue / args.steps * 1e3,
                             # the enqueue's own host work: without the time blocked on
                             # ring slots while the device is behind
                             "train_batch_enqueue_excl_ring_wait": (t_enqueue - t_wait) / args.steps * 1e3,
                             "native_step": native_step,
                             # inside the native step call (pinsage_stepper_stats): all of
                             # it, and the graph launches alone
                             **({"native_call": (st_stats["call_ns"] - st0["call_ns"]) / args.steps * 1e-6,
                                 "graph_launch": (st_stats["launch_ns"] - st0["launch_ns"]) / args.steps * 1e-6}
                                if st_stats is not None and st0 is not None else {})},
        "precompute": {"seconds": t_pre, "seconds_warm": t_pre_warm, "rng": args.precompute_rng,
                       "hops_per_s": hops / t_pre,
                       "hops_per_s_warm": hops / t_pre_warm if t_pre_warm else None,
                       "note": "wall time of precompute_neighborhoods_topt incl. the [n,100] f64+i64 "
                               "table's device-to-host copy; sampler kernels alone: "
                               "tools/precompute_probe.py"},
        "gemm_choices": gemm_choices,
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if micro:
        result["config"]["micro_batch"] = micro
        result["frontier"]["note"] = "U0/F0 of one micro-batch slice (the last outputs-only forward)"
    if cfg.get("device_build"):
        result["data"] += "; graph, features and positives drawn on the device"
        result["precompute"]["note"] = ("precompute_device_table: the model's T=50 columns of the top-100, "
                                        "built and kept in HBM")
    if rank == 0 and world == 1 and micro:
        # the reference's put_embeddings clones (n x d_in x 4 = 82 GB each)
        # and its dense [256, N_all] f64 visit matrix (205 GB) exceed the host: not run
        result["cpu_baseline"] = {"value": None, "note": "not run: the reference's per-layer put_embeddings "
                                  "clones (82 GB each) and dense visit matrices do not fit host memory"}
    elif rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(cfg, pg, feats, pos, nbhds)
        except Exception as ex:  # report, never fail the bench line
            result["cpu_baseline"] = {"error": repr(ex)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
