"""GeoBPE merge-loop benchmark (BASELINE.json metric: BPE merge iters/sec on a
PDB-pretrain-scale corpus at 1/2/4/8 MI355X).

A "step" is one BPE merge iteration (`BPE.step()`, foldingdiff/bpe.py:1792-2166)
on the BASELINE configs[2] corpus: 100k synthetic chains, lengths U{40..560}
(mean 300, ~30M residues), seed 0, bins {1: 5}; the default W + K = 10 + 990
covers the config's 1000 merges.  The prologue (thresholds, quantisation,
labels) and the initial histogram (BPE.bin) run before the timed region and are
reported separately.  Inputs are resident in HBM when the timer starts.

N > 1: one rank per GPU (RCCL); from geobpe.dist.SHARD_MIN_RANKS ranks the corpus
is row-sharded (same 100k chains in total: strong scaling) and the ranks exchange
count deltas once per iteration; below it sharding measured slower than one GPU
alone, so the ranks run as replicas (the whole corpus each, the same merges,
checked equal; the value is the job's merge rate, not N times it).
Launched by torch.distributed.run (WORLD_SIZE set: it must equal --gpus), or as
plain ``python bench.py --gpus N``: the parent then starts torch.distributed.run
with N ranks as a child process before anything touches the GPU and exits with
its status.

rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (n_chains, len_lo, len_hi, bins, merges)
    "c3": (100_000, 40, 560, 5, 1000),  # BASELINE configs[2]
    "c2": (10_000, 256, None, 5, 500),  # BASELINE configs[1]
    # BASELINE configs[4] as SURVEY §8(d) allows it: the C3 corpus, bins {1: 5}, 5000
    # merges (the multi-grid schedule cannot run in the reference's scoped mode);
    # run with --steps 4990
    "c5": (100_000, 40, 560, 5, 5000),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
LIVE = "find,commit,mid_find"  # merge-loop kernels timed live (sampled) inside the timed region
# algorithmic bytes
FIND_BYTES_PER_OCC = 136   # k_find per merged occurrence: posting entry 8, token records of p, g, b, c 64,
                           # vocab hashes of p and c 32, merge entry 16, two T entries {slot, record} 16
PLACE_BYTES_PER_OCC = 84   # k_place: merge entry 16, two T entries 16, token rewrites 28, two pk 8, two log entries 16
MIDFIND_BYTES_PER_OCC = 132  # k_mid_find: list entry 4, token records of g, p, b, c 64, vocab hashes of p and c
                             # 32, merge entry 16, two new-pair entries 16
MIDSEL_BYTES_PER_OCC = 76    # k_mid_sel's token rewrites: merge entry 16, records of a, b, c 28, two new-pair
                             # entries 16, two pk 8, (+ the appends beside the next find: two entries 8)
FIND_KREC_BYTES = 48       # k_find per key record it writes for k_commit (content hash, representative, T range)
FIND_DREC_BYTES = 8        # k_find per decrement record it writes for k_commit (key, delta)
COMMIT_KREC_BYTES = 56     # k_commit per key record: 48 read + (id, log position) 8 written
COMMIT_DREC_BYTES = 8      # per decrement record
COMMIT_KEY_BYTES = 44      # per key: table slot 8 (CAS), count 4, payload (h1, h2, len, representative) 32
PMC_WINDOWS = os.path.join(REPO, "profiles", "pmc_windows.json")
REF_TIMING = os.path.join(REPO, "profiles", "reference_cpu_timing.json")


def pmc_traffic(kernel, window_key, part="kernels"):
    """HBM bytes per launch of k_<kernel> measured by rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of THIS bench window (tools/prof_window.sh: the dispatches between the two
    k_window_mark launches), keyed by (config, warmup, steps, N); None when no pass
    of this exact window is committed -- never another window's figure."""
    try:
        with open(PMC_WINDOWS) as f:
            d = json.load(f)[window_key]
        return round(d[part][f"k_{kernel}"]["hbm_bytes_per_launch"], 1), d.get("source")
    except Exception:
        return None, None


def host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count()}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=990)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS) + ["rmsd"],
                    help="rmsd: the RMSD-partitioned mode in the README's downstream setting (bench_rmsd)")
    ap.add_argument("--rmsd-chains", type=int, default=2000, help="--config rmsd: synthetic chains")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-exchange", action="store_true",
                    help="run the multi-rank exchange (RCCL) even at world size 1: a 1-GPU rehearsal of the N>1 path")
    ap.add_argument("--cpu-budget-s", type=float, default=30.0)
    ap.add_argument("--shard-of", type=int, default=1,
                    help="rehearsal at world size 1: run rank 0's shard of an N-way row sharding (the work one "
                         "rank of N does per merge; DESIGN 5's N > 1 prediction), not the whole corpus")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: RCCL (default); gloo puts every rank on GPU 0 (a one-GPU rehearsal of the N > 1 path)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--no-replay", action="store_true", help="skip the profiled replay (per-kernel table)")
    ap.add_argument("--roofline-kernel", default="auto", help="auto: the slowest merge-loop kernel")
    ap.add_argument("--event-stride", type=int, default=0,
                    help="time every k-th launch of the merge-loop kernels in the timed region (event records "
                         "are host work: at stride 1 the host, not the GPU, sets the pace); 0 = auto: "
                         "one sample per kernel (its middle launch) below 256 steps, else max(8, steps // 32): "
                         "about 32 samples per kernel")
    ap.add_argument("--emit-merges", action="store_true",
                    help="add the merge list ([key string, count] of every merge so far) to the JSON line")
    args = ap.parse_args()
    if args.event_stride <= 0:  # (each sampled launch costs the timed region ~10 us of GPU idle)
        args.event_stride = max(1, args.steps) if args.steps < 256 else max(8, args.steps // 32)
    return args


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """``--gpus N`` (N > 1) without a launcher: start torch.distributed.run with N
    ranks as a child process (this process never touches the GPU) and return its
    exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def bench_rmsd(args):
    """--config rmsd: the RMSD-partitioned mode (geobpe/rmsd_bpe.py) in the
    README's suggested downstream setting (README.md:45, scripts/encode.sh): bins {1: 50}, histogram,
    rmsd_partition_min_size 0, --num-p 2-2:3-5:5-1:6-2:8-1, max_num_strucs 500, free bonds,
    rmsd_super_res, glue optimisation ("all", prior 0, every 10 steps).  Synthetic chains of the C3
    length law (U{40..560}, seed 0), since the PDB pretrain set is not here.  A step is one
    BPE.step() (bpe.py:1792-2166: a merge, its occurrences' k-medoids partition and assignment, the
    neighbour keys, every 10th step the glue re-optimisation); W untimed steps, then K timed.
    Per phase: initialize (thresholds, residue partitions), glue_opt_all, bin, the steps -- each
    split into the device batches (NeRF, Kabsch RMSD matrices / assignments, L-BFGS glue launches,
    timed by wrapping their entry points; each returns its result to the host) and the host
    bookkeeping (the rest)."""
    import torch
    from geobpe import glue, rmsd, synth
    from geobpe.bpe import BPE
    torch.cuda.set_device(0)
    n = args.rmsd_chains
    corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
    dev = {"s": 0.0, "calls": 0}
    for mod, names in ((rmsd, ("nerf_atoms", "nerf_packed", "geo_coords", "rmsd_matrix", "rmsd_cross")),
                       (glue, ("optimize_chains", "exit_frames"))):
        for name in names:
            f = getattr(mod, name)

            def timed(*a, _f=f, **k):
                t0 = time.perf_counter()
                r = _f(*a, **k)
                dev["s"] += time.perf_counter() - t0
                dev["calls"] += 1
                return r
            setattr(mod, name, timed)
    bpe = BPE(corpus, bins={1: 50}, bin_strategy="histogram", res_init=True, std_bonds=False,
              rmsd_partition_min_size=0, rmsd_super_res=True, num_partitions={2: 2, 3: 5, 5: 1, 6: 2, 8: 1},
              max_num_strucs=500, glue_opt=True, glue_opt_prior=0.0, glue_opt_every=10, glue_opt_method="all",
              seed=0, device=0)
    phases = {}

    def phase(name, fn):
        d0, t0 = dev["s"], time.perf_counter()
        r = fn()
        T = time.perf_counter() - t0
        phases[name] = {"s": round(T, 4), "device_s": round(dev["s"] - d0, 4), "host_s": round(T - (dev["s"] - d0), 4)}
        return r
    phase("initialize", bpe.initialize)
    phase("glue_opt_all", bpe.glue_opt_all)
    phase("bin", bpe.bin)
    phase("warmup_steps", lambda: bpe.run(args.warmup))
    d0, c0 = dev["s"], dev["calls"]
    t0 = time.perf_counter()
    done = bpe.run(args.steps)
    T = time.perf_counter() - t0
    dsec = dev["s"] - d0
    out = {
        "metric": "RMSD-mode BPE merge iters/sec (README downstream setting, synthetic chains)",
        "value": round(done / T, 3) if T > 0 else None, "unit": "merges/s", "n_gpus": 1, "steps": done,
        "warmup": args.warmup, "ms_per_step": round(1000 * T / max(done, 1), 3), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"RMSD-partitioned mode, README.md:45 setting: {n} synthetic chains, len U{{40..560}}, "
                               f"{int(corpus['row_off'][-1])} residues, bins {{1: 50}}, p_min_size 0, num_p "
                               "2-2:3-5:5-1:6-2:8-1, max_num_strucs 500, free bonds, rmsd_super_res, glue opt all "
                               f"(prior 0, every 10), steps {args.warmup + 1}..{args.warmup + done}",
                   "chains": n, "residues": int(corpus["row_off"][-1])},
        "steps_split": {"device_s": round(dsec, 4), "host_s": round(T - dsec, 4),
                        "device_share": round(dsec / T, 4) if T > 0 else None, "device_calls": dev["calls"] - c0},
        "phases": phases,
        "final": {"vocab_size": bpe.vocab_size, "merges": len(bpe._merge_log)},
    }
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.config == "rmsd":
        return bench_rmsd(args)
    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")
    if args.force_exchange:  # rehearsal of the exchange only: no tables that need per-merge counts
        args.no_profile = args.no_replay = args.no_cpu_baseline = True
        # (loopback: the rank is its own peer, its records imported by content hash -- what a rank
        # of N pays for the other ranks' records; GEOBPE_PEER_LOOPBACK=0: the one-rank protocol)
        os.environ.setdefault("GEOBPE_PEER_LOOPBACK", "1")
        if args.shard_of > 1:  # (one rank's share of an N-way run: the N-way run's regime thresholds)
            os.environ.setdefault("GEOBPE_XSHARDS", str(args.shard_of))
    world =int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if args.dist_backend == "nccl" else 0
    import torch
    import torch.distributed as dist
    from geobpe import synth
    from geobpe.dist import TorchGroup, rank_plan, shard_rows, slice_corpus
    from geobpe.engine import GeoBPEEngine

    torch.cuda.set_device(local)
    if world > 1 or args.force_exchange:
        if args.force_exchange and world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
        else:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
    n, lo, hi, B, merges = CONFIGS[args.config]
    t0 = time.time()
    lengths = synth.make_lengths(n, lo, hi, seed=0)
    corpus = synth.make_corpus(lengths, seed=0)
    R_total = int(corpus["row_off"][-1])
    t_gen = time.time() - t0
    shard = corpus
    group = None
    if args.shard_of > 1 and world == 1:  # (one rank's share of an N-way run, alone on the GPU)
        lo_r, hi_r = shard_rows(corpus["row_off"], args.shard_of)[0]
        shard = slice_corpus(corpus, lo_r, hi_r)
    plan = rank_plan(world)  # (below SHARD_MIN_RANKS the ranks are replicas: the whole corpus each)
    if (world > 1 and plan == "shard") or args.force_exchange:
        if world > 1:
            lo_r, hi_r = shard_rows(corpus["row_off"], world)[rank]
            shard = slice_corpus(corpus, lo_r, hi_r)
        group = TorchGroup(int(shard["row_off"][-1]), device=local)
        group.force = args.force_exchange
    eng = GeoBPEEngine(shard, B, device=local, group=group, max_vocab=1 << 20)
    torch.cuda.synchronize()
    t0 = time.time()
    eng.initialize()
    torch.cuda.synchronize()
    t_init = time.time() - t0
    eng.set_profiling(not args.no_profile)
    t0 = time.time()
    eng.bin()
    torch.cuda.synchronize()
    t_bin = time.time() - t0
    U0 = eng.num_keys
    bin_ms = {k: eng.kernel_ms(k)[0] for k in ("bin_sample", "pair_count", "bin_claim", "bin_assign", "finalize")}
    bin_ms = {k: v for k, v in bin_ms.items() if v > 0}
    pack_ms = eng.kernel_ms("bin_pack")[0]  # layout step for the merge loop (pk into the token records)
    eng.run(args.warmup)
    # ---- timed region: exactly K merges; HIP events around the merge-loop launches
    # (k_select carries the previous merge's k_place), on the engine's stream
    # (live events only on the kernels that can be the dominant one -- each sampled event pair
    # costs the timed region ~1 %; k_select+k_place and k_mid_sel are timed in the replay)
    eng.set_profiling(not args.no_profile, only=LIVE, stride=args.event_stride)
    st0 = eng.state()
    eng.marker(1)  # window bracket for rocprofv3 (outside the timer)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = eng.run(args.steps)
    if os.environ.get("GEOBPE_XTIME"):
        print(f"xtime: eng.run returned at +{1e6 * (time.perf_counter() - t0):.1f} us", file=sys.stderr)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    T = time.perf_counter() - t0
    eng.marker(2)
    st1 = eng.state()
    if world > 1:
        tt = torch.tensor([T], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        T = float(tt.item())
    KNAMES = ("select", "find", "commit", "mid_sel", "mid_find")
    ktimes = {k: (eng.kernel_ms(k) if not args.no_profile else (0.0, 0)) for k in KNAMES}
    merges_log = list(eng.merges)
    R_local = int(shard["row_off"][-1])
    n_ranks = dist.get_world_size() if dist.is_initialized() else 1
    rank_res = [R_local]
    if world > 1:
        rr = [None] * world
        dist.all_gather_object(rr, R_local)
        rank_res = [int(x) for x in rr]
        if plan == "replicate":  # (replicas: every rank made the same merges, or the line is void)
            mm = [None] * world
            dist.all_gather_object(mm, merges_log)
            assert all(m == merges_log for m in mm), "replica ranks made different merges"
    merge_list = eng.merge_keys() if args.emit_merges else None
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- per-kernel table: a replay of the same merges with EVERY launch timed (the timed
    # region samples every event_stride-th launch only); a second replay counts k_commit's
    # work (key records, decrement records, keys) for its algorithmic bytes -- its counters'
    # atomics slow k_commit, so no times are taken from that one
    kern, replay_avg, commit_work = {}, {}, None
    if not args.no_profile and world == 1 and not args.no_replay:
        for instrumented in (False, True):
            rep = GeoBPEEngine(shard, B, device=local, max_vocab=1 << 20)
            rep.initialize()
            rep.bin()
            rep.run(args.warmup)
            names = "commit" if instrumented else "select,find,commit,mid_sel,mid_find,tail,tail_build"
            rep.set_profiling(True, only=names)  # (every launch)
            rep.set_work_counters(instrumented)
            rep.set_hold(3000 + 60 * min(done, 64))  # (the launches queue behind a spin: no host gaps)
            rs0 = rep.state()
            rep.run(done)
            rs1 = rep.state()
            if instrumented:
                commit_work = {k: rs1[k] - rs0[k] for k in ("commit_key_records", "commit_decrement_records",
                                                            "commit_keys")}
            else:
                for k in KNAMES + ("tail", "tail_build"):
                    ms, nl = rep.kernel_ms(k)
                    if nl:
                        kern["select+place" if k == "select" else k] = {
                            "ms_total": round(ms, 4), "launches": nl, "avg_us": round(1000 * ms / nl, 3)}
                        replay_avg[k] = 1000 * ms / nl
            assert rep.merges == merges_log, "replay diverged"
            rep.close()

    # ---- roofline of the loop's kernels, from the live events of the timed region
    wkey = f"config={args.config},warmup={args.warmup},steps={args.steps},n={world}"
    window = merges_log[-done:] if done else []
    # the window's merges: the full-grid kernels ran the first n_full, the middle regime
    # (mid.h) the rest (the switch is one way); launch counts from the replay when it ran
    def _launches(k):
        kk = "select+place" if k == "select" else k
        return kern[kk]["launches"] if kk in kern else ktimes[k][1] * args.event_stride
    has_mid = bool(ktimes["mid_find"][1] or "mid_find" in kern)
    n_full = min(len(window), _launches("find")) if has_mid else len(window)
    w_full, w_mid = window[:n_full], window[n_full:]
    n_merged = sum(m[2] for m in w_full)
    mid_occ = sum(m[2] for m in w_mid)
    # the select launch of merge t places merge t - 1
    prev = merges_log[-done - 1:-1] if done and len(merges_log) > done else window
    placed = sum(m[2] for m in prev[:n_full])
    per = lambda x: x / max(len(w_full), 1)  # noqa: E731
    per_mid = lambda x: x / max(len(w_mid), 1)  # noqa: E731
    work = {"find": (FIND_BYTES_PER_OCC * per(n_merged),
                     f"{FIND_BYTES_PER_OCC} B x merged occurrences (avg {per(n_merged):.0f} per launch)"),
            "select": (PLACE_BYTES_PER_OCC * per(placed),
                       f"k_place's {PLACE_BYTES_PER_OCC} B x merged occurrences of the previous merge (avg "
                       f"{per(placed):.0f} per launch); the one-workgroup k_select beside it is not counted"),
            "commit": (None, "k_commit work counters come from the instrumented replay (--no-replay: unknown)"),
            "mid_find": (MIDFIND_BYTES_PER_OCC * per_mid(mid_occ),
                         f"{MIDFIND_BYTES_PER_OCC} B x merged occurrences (avg {per_mid(mid_occ):.0f} per launch)"),
            "mid_sel": (MIDSEL_BYTES_PER_OCC * per_mid(mid_occ),
                        f"{MIDSEL_BYTES_PER_OCC} B x merged occurrences of the previous merge (avg "
                        f"{per_mid(mid_occ):.0f} per launch); the one-workgroup select beside it is not counted")}
    if commit_work:
        cw = {k: per(v) for k, v in commit_work.items()}
        work["commit"] = (COMMIT_KREC_BYTES * cw["commit_key_records"] + COMMIT_DREC_BYTES * cw["commit_decrement_records"]
                          + COMMIT_KEY_BYTES * cw["commit_keys"],
                          f"{COMMIT_KREC_BYTES} B x key records + {COMMIT_DREC_BYTES} B x decrement records + "
                          f"{COMMIT_KEY_BYTES} B x keys (avg {cw['commit_key_records']:.0f} / "
                          f"{cw['commit_decrement_records']:.0f} / {cw['commit_keys']:.0f} per launch, counted by an "
                          f"instrumented replay of the same merges)")
    if commit_work:  # k_find also writes the key and decrement records k_commit reads
        cw = {k: per(v) for k, v in commit_work.items()}
        fb = (FIND_BYTES_PER_OCC * per(n_merged) + FIND_KREC_BYTES * cw["commit_key_records"]
              + FIND_DREC_BYTES * cw["commit_decrement_records"])
        work["find"] = (fb, f"{FIND_BYTES_PER_OCC} B x merged occurrences + {FIND_KREC_BYTES} B x key records + "
                            f"{FIND_DREC_BYTES} B x decrement records written for k_commit (avg {per(n_merged):.0f} / "
                            f"{cw['commit_key_records']:.0f} / {cw['commit_decrement_records']:.0f} per launch; the "
                            f"record counts from the instrumented replay)")
    # avg_launch_us is the replay's: every launch of the window's merges timed with HIP events
    # on the engine stream (the rocprof trace of the same window agrees, profiles/); the live
    # events of the timed region sample every event_stride-th launch and are reported beside
    # it (live_*), paired with their own merges' bytes when the window had no rebuild iteration
    per_occ = {"find": FIND_BYTES_PER_OCC, "select": PLACE_BYTES_PER_OCC, "mid_find": MIDFIND_BYTES_PER_OCC,
               "mid_sel": MIDSEL_BYTES_PER_OCC}
    src_of = {"find": w_full, "select": prev[:n_full], "mid_find": w_mid, "mid_sel": prev[n_full:]}
    no_skip = st1["nskip"] == st0["nskip"]
    roofs = {}
    for k, (ms, nl) in ktimes.items():
        live = k in LIVE.split(",") and nl > 0
        if not live and k not in replay_avg:
            continue
        bpl, note = work[k]
        live_us = 1000.0 * ms / nl if live else None
        avg_us = replay_avg.get(k, live_us)
        src = ("replay: every launch timed" if k in replay_avg
               else f"live: every {args.event_stride}th launch of the timed region, from the "
               f"{args.event_stride // 2 + 1}th (no replay)")
        live_ach = None
        if live and bpl is not None:
            lb = bpl
            if no_skip and k in per_occ:
                smp = src_of[k][args.event_stride // 2::args.event_stride][:nl]  # (the engine samples mid-stride)
                if len(smp) == nl:  # (the sampled launches' own merges)
                    lb = bpl + per_occ[k] * (sum(m[2] for m in smp) / nl - sum(m[2] for m in src_of[k]) / max(len(src_of[k]), 1))
            live_ach = lb / (live_us * 1e-6) / 1e9
        ach = bpl / (avg_us * 1e-6) / 1e9 if bpl is not None else None
        traffic, tsrc = pmc_traffic(k, wkey)  # (k_select's dispatches carry k_place)
        roofs[k] = {"kernel": {"select": "k_select+k_place", "mid_sel": "k_mid_sel"}.get(k, f"k_{k}"), "bound": "hbm",
                    "achieved": round(ach, 2) if ach else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 5) if ach else None,
                    "traffic": traffic, "traffic_source": tsrc, "traffic_window": wkey,
                    "traffic_frac_of_algorithmic": round(traffic / bpl, 2) if traffic and bpl else None,
                    "bytes_per_launch": round(bpl, 1) if bpl is not None else None,
                    "avg_launch_us": round(avg_us, 3), "avg_source": src,
                    "ms_total": kern.get("select+place" if k == "select" else k, {}).get("ms_total"),
                    "algorithmic_bytes": note,
                    "live_avg_launch_us": round(live_us, 3) if live else None,
                    "live_launches_timed": nl if live else 0, "event_stride": args.event_stride if live else None,
                    "live_achieved": round(live_ach, 2) if live_ach else None}
    if args.roofline_kernel == "auto":
        # the dominant kernel: the most total time over the window's launches (replay), among
        # the kernels that can dominate (k_select+k_place rides with a one-workgroup select)
        cand = [k for k in roofs if k in LIVE.split(",")] or list(roofs)
        tot = lambda k: (roofs[k]["ms_total"] if roofs[k]["ms_total"] is not None  # noqa: E731
                         else roofs[k]["avg_launch_us"] * _launches(k) / 1000.0)
        dom = max(cand, key=tot) if cand else None
    else:
        dom = args.roofline_kernel if args.roofline_kernel in roofs else None
    roofline = roofs.get(dom) if dom else None
    roofline_other = {k: v for k, v in roofs.items() if k != dom}
    # the full content-keyed pair-count pass (BPE.bin) at iteration 0: SURVEY §8(d)
    # B_count = 20*T_live + 4*U_live with T = residues
    pair_count = None
    if bin_ms.get("pair_count"):
        bc = 20.0 * R_local + 4.0 * U0
        t_pass = sum(bin_ms.values()) / 1000.0
        t_count = bin_ms["pair_count"] / 1000.0
        dense = "bin_claim" in bin_ms
        ctraffic = pmc_traffic("bin_count" if dense else "pairs_all", wkey, "pre_kernels")[0]
        pair_count = {
            "bytes": bc, "T0": R_local, "U0": U0,
            "count_kernel": {"kernel": "k_bin_count" if dense else "k_pairs_all",
                             "time_us": round(t_count * 1e6, 2), "achieved_GBs": round(bc / t_count / 1e9, 1),
                             "frac": round(bc / t_count / 1e9 / HBM_PEAK_GBS, 4),
                             "frac_basis": "SURVEY 8(d) B_count = 20*T + 4*U bytes",
                             "traffic": ctraffic,
                             # the counters' own bytes (FETCH + WRITE of this launch) over the same time
                             "traffic_frac": (round(ctraffic / t_count / 1e9 / HBM_PEAK_GBS, 4) if ctraffic else None)},
            "pass": {"kernels": ("k_bin_sample+k_bin_rank+k_bin_flag+k_bin_precube | k_bin_count | k_bin_reduce | "
                                 "k_bin_ool_stage+k_bin_ool_claim+k_bin_ool_fix") if dense else "k_pairs_all+k_finalize",
                     "time_us": round(t_pass * 1e6, 2), "achieved_GBs": round(bc / t_pass / 1e9, 1),
                     "frac": round(bc / t_pass / 1e9 / HBM_PEAK_GBS, 4),
                     "ms": {k: round(v, 4) for k, v in bin_ms.items()}},
            "layout_pack_us": round(pack_ms * 1000, 2),
            # the merge loop's token records: k_bin_count writes them itself since round 5
            # (FUSE_PACK: pack_us 0); before, k_pack copied pk into them after the pass
            "pack_us": round(pack_ms * 1000, 2),
            "pack_fused": pack_ms == 0,
            "pass_and_pack": {"time_us": round(t_pass * 1e6 + pack_ms * 1000, 2),
                              "frac": round(bc / (t_pass + pack_ms / 1000.0) / 1e9 / HBM_PEAK_GBS, 4)},
        }

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(corpus, B, args.warmup, args.steps, args.cpu_budget_s)
        cpu["host"] = host_cpu()
        cpu["reference"] = reference_estimate(window)

    value = done / T if T > 0 else 0.0
    out = {
        "metric": "BPE merge iters/sec on PDB-pretrain-scale corpus",
        "value": round(value, 2),
        "unit": "merges/s",
        "n_gpus": n_ranks,
        "steps": done,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * T / max(done, 1), 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": (f"BASELINE configs[{ {'c3': 2, 'c5': 4}[args.config]}]"
                                + (" (bins {1: 5} form, SURVEY 8(d))" if args.config == "c5" else "")
                                + f": {n} synthetic chains, len U{{{lo}..{hi}}}, {R_total} residues, "
                                f"bins {{1: {B}}}, merges {args.warmup + 1}..{args.warmup + done}")
                   if args.config in ("c3", "c5") else f"BASELINE configs[1]: {n}x{lo}, bins {{1: {B}}}",
                   "chains": n, "residues": R_total, "bins": B,
                   "parallelism": f"{'replicas' if world > 1 and plan == 'replicate' else 'rows'}{world}",
                   "rank_residues": rank_res, "backend": (args.dist_backend if world > 1 else None),
                   **({"shard_of": args.shard_of} if args.shard_of > 1 else {}),
                   **({"exchange": "rehearsal (world 1)" + (", all-gather" if os.environ.get("GEOBPE_PEER") == "0"
                                                             else ", peer" + (", loopback" if os.environ.get(
                                                                 "GEOBPE_PEER_LOOPBACK") == "1" else ""))}
                      if args.force_exchange else {})},
        "roofline": roofline,
        "roofline_other": roofline_other,
        "cpu_baseline": cpu,
        "pair_count_pass": pair_count,
        "kernels": kern,
        "prologue_s": {"generate": round(t_gen, 3), "initialize": round(t_init, 3), "bin": round(t_bin, 3)},
        "final": {"vocab": eng.vocab_count, "keys": eng.num_keys},
    }
    if merge_list is not None:
        out["merge_list"] = merge_list
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    if world > 1 or args.force_exchange:
        dist.destroy_process_group()


def reference_estimate(window):
    """The reference Python's own cost (foldingdiff/bpe.py BPE.step, timed in the build
    container by tools/ref_timing.py on C3 subsets: ms per merged occurrence) applied
    to this window's merged occurrences -- context, not a measurement on this host."""
    try:
        with open(REF_TIMING) as f:
            rt = json.load(f)
    except (OSError, ValueError):
        return None
    runs = rt["runs"]
    ms_occ = max(r["ms_per_merged_occurrence"] for r in runs)
    occ = sum(m[2] for m in window) / max(len(window), 1)
    return {"value": round(1000.0 / (ms_occ * occ), 6) if occ else None, "unit": "merges/s",
            "ms_per_merged_occurrence": ms_occ, "merged_occurrences_per_merge": round(occ, 1),
            "cores": 1, "host": f"build container, {rt.get('cpus', '?')} vCPU (not the GPU box)",
            "kind": "reference", "sample": f"{rt['generator']}: step() on the first "
            + "/".join(str(r["chains"]) for r in runs) + " chains of the C3 corpus, "
            + f"{rt.get('merges_timed', '?')} merges each; slowest per-occurrence cost used"}


def cpu_baseline(corpus, B, warmup, steps, budget_s):
    """The CPU oracle (C restatement of the reference loop, 1 core) on the same
    corpus and the same merge window, stopped after ``budget_s`` of timed work."""
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"error": repr(e)}
    o = oracle.OracleBPE(corpus, B).initialize()
    o.bin()
    for _ in range(warmup):
        o.step_fast()
    t0 = time.perf_counter()
    done = 0
    while done < steps:
        if o.step_fast() is None:
            break
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    T = time.perf_counter() - t0
    return {"value": round(done / T, 2), "unit": "merges/s", "cores": 1, "kind": "port",
            "sample": f"oracle/geobpe_oracle.c on the same corpus, merges {warmup + 1}..{warmup + done} "
                      f"({T:.1f} s of single-core work)"}


if __name__ == "__main__":
    main()
