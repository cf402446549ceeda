"""bench.py -- genotyped reference positions/s of the MI355X SNV pileup path.

Workload (BASELINE.json configs[1]): yeast whole genome (sacCer3 contig names/lengths,
12,157,105 bp, synthetic bases) at 30x, 150 bp single-end synthetic reads, one sample.
A step = one pass of the hot path over the whole genome with the pileup resident in HBM:
k_tile_pileup (tile scan + hom-ref bounds) + k_posterior (exact tally, posterior and call of the
undecided candidates) + ko_* (position order) + D2H of the called sites + host mapping to
(sequence, position) (libngsep_amd.so, ngsep_submit_staged / ngsep_collect_staged, two passes in
flight so one pass's copies overlap the next pass's kernels).  N>1: one process per GPU, each rank owns its own
synthetic genome (seed 2+rank) -- windows shard with no data-path collective ("weak").

--config multisample (BASELINE.json configs[4], MultisampleVariantsDetector): 200 samples at 10x
(population SNVs in HWE), one rank = one contig shard of the 8-GPU split (default chrIV, the largest
yeast contig, ~1/8 of the genome); a step = KTM (per-sample tile scan) + KPM (population
genotyping) + D2H of the sites and every sample's call.

Prints one JSON line (rank 0).  --gpus N under torch.distributed.run for N>1.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "tools", "synth"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "genotyped ref positions/sec on 30x synthetic BAM; 1/2/4/8 GPU scaling"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(depth: float, seed: int, n_contigs: int):
    """The oracle (single-thread C restatement of the reference) on a bounded sample of the same
    workload: the first n_contigs yeast contigs at the same depth, SAM text -> VCF."""
    import ngsep_oracle
    import pysynth
    syn = pysynth.Synth(genome=pysynth.YEAST, depth=depth, seed=seed, n_contigs=n_contigs)
    names = [n for n, _ in syn.contigs()]
    with tempfile.TemporaryDirectory() as d:
        fa, sam, _ = syn.write(os.path.join(d, "cpu"))
        st = ngsep_oracle.run_ssvd(fa, sam, os.path.join(d, "cpu.vcf"))
    syn.close()
    return {
        "value": st.positions_genotyped / st.seconds,
        "unit": "positions/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle (C restatement, SAM->VCF incl. parsing) on yeast {names[0]}..{names[-1]} "
                  f"({st.positions_genotyped} positions) at {depth:g}x, {st.seconds:.2f} s",
    }


def cpu_baseline_mvd(samples: int, depth: float, length: int = 20000):
    """The oracle's MultisampleVariantsDetector (single thread) on a bounded sample: the same
    population model on a 20 kb contig."""
    import ngsep_oracle
    import pysynth
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=length, depth=depth, seed=5, n_samples=samples)
    with tempfile.TemporaryDirectory() as d:
        fa, sam, _ = syn.write(os.path.join(d, "cpu"))
        st = ngsep_oracle.run_mvd(fa, sam, os.path.join(d, "cpu.vcf"))
    syn.close()
    return {
        "value": st.positions_genotyped / st.seconds,
        "unit": "positions/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle MultisampleVariantsDetector (C restatement, SAM->VCF) on {samples} samples x "
                  f"{length} bp at {depth:g}x ({st.positions_genotyped} positions), {st.seconds:.2f} s",
    }


def cold_passes(sess, n: int = 5):
    """Passes with the Infinity Cache (256 MiB) flushed first: a 1 GiB device fill before each (HIP
    runtime through ctypes), so the scan reads its layout from HBM (steady-state passes re-read a
    bit-plane pile that fits on-die)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    size = ctypes.c_size_t(1 << 30)
    buf = ctypes.c_void_p()
    if hip.hipMalloc(ctypes.byref(buf), size) != 0:
        return None
    wall, scan = [], []
    try:
        for i in range(n):
            if hip.hipMemset(buf, ctypes.c_int(i & 0xFF), size) != 0 or hip.hipDeviceSynchronize() != 0:
                return None
            t = time.perf_counter()
            sess.run_staged()
            wall.append((time.perf_counter() - t) * 1e3)
            scan.append(sess.stats().scan_ms)
    finally:
        hip.hipFree(buf)
    return {"passes": n, "pass_ms": sum(wall) / n, "scan_kernel_ms": sum(scan) / n,
            "note": "1 GiB device fill before each pass (Infinity Cache flushed); synchronous submit+collect"}


def load_traffic(workload_key: str):
    """Per-launch HBM bytes of the scan kernel from the committed PMC passes (profiles/pmc_traffic*.json,
    one file per workload), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload_key") == workload_key:
            return d.get("bytes_per_launch")
    return None


def bench_coverage(args):
    """--config coverage: CoverageStats (CoverageStatisticsCalculator) on the same
    yeast 30x reads, resident in HBM; a step = one kc_tile_hist pass + D2H of the histograms (1 GPU)."""
    import pysynth
    from ngsepcore_amd import GpuPileupSession, default_params
    syn = pysynth.Synth(genome=pysynth.YEAST, depth=args.depth, seed=2)
    p = default_params()
    p.coverage_stats, p.process_secondary, p.max_alns_per_start = 1, 1, 100
    sess = GpuPileupSession(p)
    for name, seq in syn.contigs():
        sess.set_reference(name, seq)
    sess.stage(syn.batch())
    sess.stage_finish()
    syn.close()
    st = sess.stats()
    for _ in range(args.warmup):
        sess.run_staged()
    ks = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sess.run_staged()
        ks.append(sess.stats().scan_ms)
    elapsed = time.perf_counter() - t0
    sess.release_staged()
    sess.close()
    k_ms = sum(ks) / len(ks)
    # algorithmic bytes per launch: 12 B per admitted read (global first + span|unique) + the histograms
    alg = 12 * st.alignments_admitted + 16 * (p.max_coverage + 1)
    ach = alg / (k_ms * 1e-3) / 1e9
    print(json.dumps({
        "metric": "covered positions/sec (CoverageStats histograms), yeast 30x synthetic", "value": st.positions_genotyped * args.steps / elapsed,
        "unit": "positions/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int32/u64", "data": "synthetic (seeded generator); admitted reads resident in HBM",
        "config": {"workload": "CoverageStats on yeast whole genome 30x synthetic 150 bp SE", "positions_per_gpu": st.positions_genotyped,
                   "reads_per_gpu": int(st.alignments_admitted), "max_coverage": p.max_coverage},
        "roofline": {"bound": "hbm", "kernel": "kc_tile_hist", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": None, "alg_bytes_per_launch": alg, "kernel_avg_ms": k_ms,
                     "note": "LDS-bound (difference array + workgroup scan over 4096 positions per tile), not HBM-bound"},
    }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--no-cold", action="store_true", help="skip the cache-flushed passes")
    ap.add_argument("--genome", default="yeast", choices=["yeast", "human_chr20"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-contigs", type=int, default=4)
    ap.add_argument("--config", default="single", choices=["single", "multisample", "coverage"])
    ap.add_argument("--samples", type=int, default=200)
    ap.add_argument("--contig-first", type=int, default=3, help="multisample: first yeast contig of the shard")
    ap.add_argument("--n-contigs", type=int, default=1, help="multisample: contigs in the shard")
    args = ap.parse_args()
    if args.config == "multisample" and args.depth == 30.0:
        args.depth = 10.0

    if args.config == "coverage":
        return bench_coverage(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend="nccl")
        dist = tdist

    import pysynth
    from ngsepcore_amd import GpuPileupSession, default_params

    seed = 2 + rank
    t0 = time.time()
    multi = args.config == "multisample"
    if multi:
        seed = 5
        syn = pysynth.Synth(genome=pysynth.YEAST, depth=args.depth, seed=seed, n_samples=args.samples,
                            contig_first=args.contig_first + rank, n_contigs=args.n_contigs)
        names = [n for n, _ in syn.contigs()]
        workload = (f"MultisampleVariantsDetector: {args.samples} synthetic yeast samples at {args.depth:g}x, "
                    f"shard {'+'.join(names)} (one GPU's contig shard of the 8-GPU split)")
    elif args.genome == "yeast":
        syn = pysynth.Synth(genome=pysynth.YEAST, depth=args.depth, seed=seed)
        workload = "yeast whole genome (sacCer3 names/lengths, 12,157,105 bp) 30x synthetic 150 bp SE"
    else:
        syn = pysynth.Synth(genome=pysynth.HUMAN, depth=args.depth, seed=3 + rank, contig_first=19, n_contigs=1)
        workload = "human chr20 (64,444,167 bp) 30x synthetic 150 bp SE"
    t_gen = time.time() - t0
    params = default_params()
    if multi:
        params.multisample = 1
    sess = GpuPileupSession(params, device=local_rank)
    if multi:
        n = max(1, syn.params.n_samples)
        sess.set_samples([(f"S{k:03d}", f"S{k:03d}") for k in range(n)])
    for name, seq in syn.contigs():
        sess.set_reference(name, seq)
    t1 = time.time()
    sess.stage(syn.batch())
    sess.stage_finish()
    t_stage = time.time() - t1
    n_reads_in = syn.n_reads
    syn.close()
    st = sess.stats()
    positions = st.positions_genotyped
    log(f"[rank {rank}] generated in {t_gen:.1f}s, staged {st.alignments_admitted} reads "
        f"({st.read_bases} read bases, {st.slot_bytes} slot bytes) over {positions} positions in {t_stage:.1f}s")

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        sess.run_staged()
    barrier()
    scan_ms, geno_ms, dev_ms = [], [], []
    t_start = time.perf_counter()
    # a stream of passes, two in flight: pass k+1's kernels run while pass k's records are copied
    # back and mapped (ngsep_submit_staged / ngsep_collect_staged); every pass is collected
    sess.submit_staged()
    t_sub = t_col = 0.0
    for k in range(args.steps):
        t1 = time.perf_counter()
        if k + 1 < args.steps:
            sess.submit_staged()
        t2 = time.perf_counter()
        sess.collect_staged()
        t3 = time.perf_counter()
        t_sub += t2 - t1
        t_col += t3 - t2
        s = sess.stats()
        scan_ms.append(s.scan_ms)
        geno_ms.append(s.genotype_ms)
        dev_ms.append(s.kernel_ms)
    barrier()
    elapsed = time.perf_counter() - t_start
    st = sess.stats()
    if os.environ.get("NGSEP_PROBE_HOST"):     # diagnostics: host cost of a collect whose pass is done
        tc = ts = tt = 0.0
        for _ in range(20):
            t1 = time.perf_counter()
            sess.submit_staged()
            t2 = time.perf_counter()
            time.sleep(0.003)
            t3 = time.perf_counter()
            sess.collect_staged()
            t4 = time.perf_counter()
            sess.stats()
            t5 = time.perf_counter()
            ts += t2 - t1
            tc += t4 - t3
            tt += t5 - t4
        log(f"[rank {rank}] idle-GPU host cost: submit {ts / 20 * 1e3:.4f} ms, collect {tc / 20 * 1e3:.4f} ms, stats {tt / 20 * 1e3:.4f} ms")
    n_sites = st.sites_called
    log(f"[rank {rank}] host per pass: submit {1e3 * t_sub / args.steps:.4f} ms, collect (incl. wait) {1e3 * t_col / args.steps:.4f} ms")
    log(f"[rank {rank}] tile {st.tile_positions} positions (max {st.tile_rows_max} rows), pile {st.pile_bytes} B, "
        f"slot {st.slot_size} B, {st.candidates} candidates, {st.exact_bound_passes} exact-bound passes, "
        f"{st.hard_sites} needed the exact tally + posterior")
    cold = cold_passes(sess) if world == 1 and not args.no_cold else None
    sess.release_staged()
    sess.close()

    if dist is not None:
        import torch
        t = torch.tensor([elapsed, float(positions)], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        total_positions = float(t[1])
    else:
        total_positions = float(positions)

    if rank == 0:
        steps = args.steps
        value = total_positions * steps / elapsed
        k_avg_ms = sum(scan_ms) / len(scan_ms)
        post_avg_ms = (sum(geno_ms) / len(geno_ms)) if max(geno_ms, default=0) > 0 else None
        # algorithmic bytes per k_tile_pileup launch: 1 B per projected read base,
        # 1 B reference per genotyped position, 16 B read header per admitted read
        alg_bytes = st.read_bases + positions + 16 * st.alignments_admitted
        achieved = alg_bytes / (k_avg_ms * 1e-3) / 1e9 if k_avg_ms > 0 else None
        workload_key = (f"multisample{args.samples}:{args.depth:g}x:contig{args.contig_first}" if multi
                        else f"{args.genome}:{args.depth:g}x:seed{seed}")
        traffic = load_traffic(workload_key)
        planes = not multi and st.tile_positions in (128, 256, 512) and not os.environ.get("NGSEP_NO_PLANES")
        scan_kernel = ("k_tile_pileup_multi" if multi else
                       f"k_tile_planes<{st.tile_positions // 32}>" if planes else "k_tile_pileup<0>")
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "positions/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8,f64",
            "data": "synthetic (seeded generator, SURVEY.md 8(d)); read SoA resident in HBM",
            "config": {
                "workload": workload,
                "positions_per_gpu": positions,
                "reads_per_gpu": int(st.alignments_admitted),
                "read_bases_per_gpu": int(st.read_bases),
                "sites_called_per_gpu": int(n_sites),
                "candidates_per_gpu": int(st.candidates),
                "exact_sites_per_gpu": int(st.hard_sites),
                "pile_bytes_per_gpu": int(st.pile_bytes),
                "tile_positions": int(st.tile_positions),
                "parallelism": f"dp{world} (independent genomic windows per GPU, no collective)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": scan_kernel,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes,
                "kernel_avg_ms": k_avg_ms,
                # achieved counts the algorithmic bytes; the bit-plane scan moves a quarter
                # of them, so its HBM rate is traffic / time
                "traffic_rate_GBs": (traffic / (k_avg_ms * 1e-3) / 1e9) if traffic and k_avg_ms > 0 else None,
                "cold": cold,
                # KP is timed only with NGSEP_TIME_POSTERIOR=1 (its event costs ~7 us of pipeline gap)
                "posterior_kernel_avg_ms": post_avg_ms,
            },
            "kernel_positions_per_s": (total_positions / ((k_avg_ms + post_avg_ms) * 1e-3)) if post_avg_ms else None,
        }
        if multi:
            line["config"]["samples"] = args.samples
            line["config"]["sample_calls_per_step"] = int(n_sites) * args.samples
        if not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = (cpu_baseline_mvd(args.samples, args.depth) if multi
                                        else cpu_baseline(args.depth, 2, args.cpu_contigs))
            except Exception as e:  # the baseline is reported, never required
                line["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
