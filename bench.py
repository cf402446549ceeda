"""bench.py -- genotyped reference positions/s of the MI355X SNV pileup path.

Workload (BASELINE.json configs[2], the largest single-GPU configuration and the one the roofline is
quoted on): human chr20 (64,444,167 bp, synthetic bases) at 30x, 150 bp single-end synthetic reads, one
sample.  The host packer's output -- the admitted reads' reference-projected code bytes (1 B per read base,
pending-list order) in 64-read groups, 8-byte headers, reference codes -- is resident
in HBM before the timed region; a step = one pass of the hot path over it: KL (per-position coverage, the
other-allele / exception tallies and the count bound straight from the read bytes, the survivors' columns
gathered) + KP (exact tally, posterior and call of the survivors) + KO (position order, (sequence,
position) mapping) + D2H of the called sites + the host collect (libngsep_amd.so ngsep_submit_staged /
ngsep_collect_staged, two passes in flight).

Beside the resident rate the line carries:
  * roofline   -- SURVEY.md 8(d)'s algorithmic bytes per launch (1 B per read base + 1 B of reference per
                  genotyped position + 16 B per read) / KL's average launch time from HIP events bound to
                  its dispatch; `bytes_moved_per_launch` = what KL actually reads (units incl. padding,
                  8-B headers, group and block tables, reference codes); `traffic` = HBM bytes per launch
                  from the committed rocprofv3 PMC passes (profiles/pmc_traffic*.json);
  * end_to_end -- BAM on disk -> VCF on disk through ngsep_call_bam (path B: BGZF decode, admission,
                  projection, layout, H2D, kernels, VCF), wall time and positions/s;
  * cpu_baseline -- the oracle (C restatement of the reference, SAM -> VCF) on a bounded sample of the
                  same workload, single-thread and one process per core.

--gpus N > 1: one process per GPU (spawned here under torch.distributed.run when WORLD_SIZE is unset), the same
workload per GPU as at N = 1 (the default chr20: each rank its own chr20-sized genome, seed 3 + rank -- independent
genomic windows, no data-path collective, "weak"), so the 1/2/4/8 values divide: value = every rank's positions x
steps / the slowest rank's time.  At N > 1 the line also carries the CPU baseline (rank 0, before any GPU call), the
end-to-end leg on every rank (its own BAM -> VCF, slowest rank, positions summed) and a strong-scaling leg
(sharded_end_to_end: ONE chr20 BAM cut into exact windows over the ranks).  --config wgs: BASELINE.json configs[3],
the GRCh38 sequences (30x) split over the ranks by sharding.assign_contigs (the genome is fixed: "strong"; at N = 1
the whole genome on one GPU, --wgs-shard picks one GPU's shard of an 8-way split).
--config yeast: configs[1].  --config multisample: configs[4] (one GPU's contig shard of the 200-sample
population).  --config coverage: CoverageStats on yeast 30x.

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
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
HUMAN_CHR20 = 19               # index of chr20 in the synthetic GRCh38 table


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_cores() -> int:
    """The CPU share of this process (the same rule as the library's host_threads(), engine.hpp): NGSEP_THREADS; else
    the affinity mask divided among the node's ranks (LOCAL_WORLD_SIZE), at most OMP_NUM_THREADS when that is above 1
    (the GPU box's share, 16; torch.distributed.run's default of 1 is not a share)."""
    v = os.environ.get("NGSEP_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return min(int(v), 64)
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    share = max(1, cores // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 1:
        share = min(share, int(omp))
    return min(share, 64)


# ------------------------------------------------------------------------------------------------
# CPU baseline: the oracle on a bounded sample of the same workload (before any GPU call)
# ------------------------------------------------------------------------------------------------
def _write_piece(d, k, genome, contig_first, trunc, depth, seed):
    import pysynth
    syn = pysynth.Synth(genome=genome, contig_first=contig_first, n_contigs=1, trunc_len=trunc, depth=depth,
                        seed=seed, rng_per_contig=1)
    fa, sam, _ = syn.write(os.path.join(d, f"piece{k}"))
    syn.close()
    return fa, sam


def cpu_baseline(genome: int, contig_first: int, depth: float, trunc: int, seed: int):
    """Single thread: the oracle (SAM text -> VCF, like the Java path incl. reading its input) on the first
    `trunc` bp of the workload's sequence.  All cores: one oracle process per core, each on its own
    `trunc`-bp piece (independent synthetic sequences), wall time over the pool."""
    import ngsep_oracle
    cli = os.path.join(ROOT, "oracle", "build", "ngsep_oracle")
    cores = cpu_cores()
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fa, sam = _write_piece(d, 0, genome, contig_first, trunc, depth, seed)
        st = ngsep_oracle.run_ssvd(fa, sam, os.path.join(d, "one.vcf"))
        one = {"value": st.positions_genotyped / st.seconds, "cores": 1,
               "sample": f"{st.positions_genotyped} positions ({trunc / 1e6:g} Mb of the workload's sequence) at "
                         f"{depth:g}x, {st.seconds:.2f} s"}
        pieces = [(fa, sam)] + [_write_piece(d, k, genome, contig_first, trunc, depth, seed + 1000 * k)
                                for k in range(1, cores)]
        t0 = time.perf_counter()
        procs = [subprocess.Popen([cli, "-r", f, "-i", s, "-o", os.path.join(d, f"all{k}")],
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
                 for k, (f, s) in enumerate(pieces)]
        positions = 0
        for p in procs:
            _, err = p.communicate()
            if p.returncode != 0:
                raise RuntimeError(f"oracle failed: {err}")
            positions += int(err.split("positions=")[1].split()[0])
        wall = time.perf_counter() - t0
    out = {"value": positions / wall, "unit": "positions/s", "cores": cores, "kind": "port",
           "sample": f"oracle (C restatement of the reference, SAM -> VCF incl. parsing), {cores} processes x "
                     f"{trunc / 1e6:g} Mb synthetic pieces at {depth:g}x ({positions} positions) in {wall:.2f} s wall",
           "single_thread": one}
    return out


def cpu_baseline_mvd(samples: int, depth: float, length: int = 20000):
    """The oracle's MultisampleVariantsDetector on a bounded sample (the same population model on 20 kb contigs):
    single thread, and one oracle process per core, each on its own contig (independent seeds), wall time over
    the pool."""
    import ngsep_oracle
    import pysynth
    cli = os.path.join(ROOT, "oracle", "build", "ngsep_oracle")
    cores = cpu_cores()

    def piece(d, k):
        syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=length, depth=depth, seed=5 + 1000 * k, n_samples=samples)
        fa, sam, _ = syn.write(os.path.join(d, f"cpu{k}"))
        syn.close()
        return fa, sam

    with tempfile.TemporaryDirectory() as d:
        pieces = [piece(d, k) for k in range(cores)]
        st = ngsep_oracle.run_mvd(pieces[0][0], pieces[0][1], os.path.join(d, "cpu.vcf"))
        one = {"value": st.positions_genotyped / st.seconds, "cores": 1,
               "sample": f"{samples} samples x {length} bp at {depth:g}x ({st.positions_genotyped} positions), "
                         f"{st.seconds:.2f} s"}
        t0 = time.perf_counter()
        procs = [subprocess.Popen([cli, "MultisampleVariantsDetector", "-r", f, "-o", os.path.join(d, f"all{k}.vcf"), s],
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
                 for k, (f, s) in enumerate(pieces)]
        positions = 0
        for p in procs:
            _, err = p.communicate()
            if p.returncode != 0:
                raise RuntimeError(f"oracle failed: {err}")
            positions += int(err.split("positions=")[1].split()[0])
        wall = time.perf_counter() - t0
    return {
        "value": positions / wall,
        "unit": "positions/s",
        "cores": cores,
        "kind": "port",
        "sample": f"oracle MultisampleVariantsDetector (C restatement, SAM -> VCF), {cores} processes x {samples} "
                  f"samples x {length} bp at {depth:g}x ({positions} positions) in {wall:.2f} s wall",
        "single_thread": one,
    }


# ------------------------------------------------------------------------------------------------
# measurement helpers
# ------------------------------------------------------------------------------------------------
def cold_passes(sess, n: int = 5):
    """Passes with the Infinity Cache (256 MiB) flushed first: a 1 GiB device fill before each (HIP
    runtime through ctypes), so the scan reads its layout from HBM."""
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
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json")), reverse=True):   # newest tag first
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload_key") == workload_key:
            return d.get("bytes_per_launch")
    return None


def end_to_end(fa: str, bam: str, device: int):
    """BAM on disk -> VCF on disk: SingleSampleVariantsDetector.findSNVS through ngsep_call_bam in a fresh
    context (decode, admission, projection, layout, H2D, kernels, VCF writing), wall time."""
    from ngsepcore_amd import GpuPileupSession
    out = os.path.join(os.path.dirname(bam), "e2e.vcf")
    with GpuPileupSession(device=device) as s:
        t0 = time.perf_counter()
        s.load_fasta(fa)
        t1 = time.perf_counter()
        s.processFile(bam, out)
        t2 = time.perf_counter()
        st = s.stats()
    n_rec = sum(1 for l in open(out) if not l.startswith("#"))
    return {"wall_s": t2 - t0, "fasta_s": t1 - t0, "call_bam_s": t2 - t1,
            "positions": int(st.positions_genotyped), "value": st.positions_genotyped / (t2 - t0),
            "unit": "positions/s", "vcf_records": n_rec, "bam_bytes": os.path.getsize(bam),
            "realign_regions": int(st.realign_regions), "realign_replay_ms": float(st.realign_ms),
            "phases_ms": {"realign_replay": float(st.realign_ms), "keep_raw": float(st.keep_raw_ms),
                          "region_setup": float(st.region_setup_ms), "region_device": float(st.region_device_ms),
                          "region_merge": float(st.region_merge_ms), "window_wait": float(st.window_wait_ms),
                          "region_gather": float(st.region_gather_ms),
                          "layout": float(st.layout_ms), "upload": float(st.upload_ms),
                          "note": "host wall times summed over the windows (the replays, the regions' device run and "
                                  "merge run on the window worker, beside the reader); window_wait: the reader joining "
                                  "the worker"},
            "note": "ngsep_call_bam: BAM on disk -> VCF on disk incl. FASTA load; host threads "
                    f"{os.environ.get('NGSEP_THREADS') or cpu_cores()}"}


def end_to_end_population(fa: str, bams, device: int):
    """BAM files on disk -> population VCF on disk: MultisampleVariantsDetector.run through
    ngsep_call_population_bams in a fresh context (merge of the sample BAMs in the generator's order, decode,
    admission, population layout, H2D, KLM/KPM, VCF writing), wall time."""
    from ngsepcore_amd.discovery import MultisampleVariantsDetector
    out = os.path.join(os.path.dirname(fa), "e2e_pop.vcf")
    mvd = MultisampleVariantsDetector()
    mvd.device = device
    mvd.setGenome(fa)
    mvd.setOutFilename(out)
    t0 = time.perf_counter()
    s = mvd.run(list(bams))
    t1 = time.perf_counter()
    st = s.stats()
    s.close()
    n_rec = sum(1 for l in open(out) if not l.startswith("#"))
    return {"wall_s": t1 - t0, "positions": int(st.positions_genotyped), "value": st.positions_genotyped / (t1 - t0),
            "unit": "positions/s", "vcf_records": n_rec, "bams": len(bams),
            "bam_bytes": sum(os.path.getsize(b) for b in bams),
            "note": "ngsep_call_population_bams: sample BAMs on disk -> population VCF on disk incl. FASTA load; "
                    f"host threads {os.environ.get('NGSEP_THREADS') or cpu_cores()}"}


def sharded_end_to_end(args, dist, rank, local_rank, backend):
    """--gpus N > 1: configs[2]'s chr20 BAM -> VCF through the product's own sharding (sharding.call_bam_sharded: exact
    windows from ngsep_clean_cut taken by the ranks from the process group's shared queue, each window a BAI region run
    on the rank's GPU, the blocks merged on rank 0), wall time from a barrier to a barrier, max over ranks.  Rank 0 writes
    the BAM (untimed) into a directory every rank of the node reads."""
    import pysynth
    import torch
    from ngsepcore_amd.sharding import call_bam_sharded
    box = [None]
    if rank == 0:
        tmp = tempfile.mkdtemp(prefix="ngsep_sharded_")
        syn = pysynth.Synth(genome=pysynth.HUMAN, depth=args.depth, seed=3, contig_first=HUMAN_CHR20, n_contigs=1,
                            rng_per_contig=1)
        fa, bam = os.path.join(tmp, "chr20.fa"), os.path.join(tmp, "chr20.bam")
        pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
        pysynth.lib().ngs_synth_write_bam(syn.h, bam.encode())
        seq_len = sum(len(x) for _, x in syn.contigs())
        syn.close()
        box = [(tmp, fa, bam, seq_len)]
    dist.broadcast_object_list(box, src=0)
    tmp, fa, bam, seq_len = box[0]
    dev = "cuda" if backend == "nccl" else "cpu"
    work = {}
    dist.barrier()
    t0 = time.perf_counter()
    call_bam_sharded(fa, bam, os.path.join(tmp, "sharded.vcf"), dist=dist, device=local_rank, window=4 << 20, work=work)
    dist.barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall, float(work.get("windows", 0)), float(work.get("positions", 0))], dtype=torch.float64, device=dev)
    mx = t[:1].clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = t[1:].clone()
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    out = None
    if rank == 0:
        n_rec = sum(1 for l in open(os.path.join(tmp, "sharded.vcf")) if not l.startswith("#"))
        w = float(mx[0])
        out = {"wall_s": w, "value": seq_len / w, "unit": "positions/s", "sequence_bp": seq_len, "vcf_records": n_rec,
               "windows": int(sm[0]), "region_positions": int(sm[1]), "bam_bytes": os.path.getsize(bam),
               "note": f"sharding.call_bam_sharded over {dist.get_world_size()} ranks: chr20 30x BAM on local disk -> "
                       "merged VCF, 4 Mb windows cut by ngsep_clean_cut from the process group's shared queue, BAI region "
                       "reads (strong scaling: one sequence over the ranks); value = the sequence's positions (every one "
                       "covered at 30x) / wall; region_positions counts the windows' lead-ins too; host threads per rank "
                       f"{os.environ.get('NGSEP_THREADS') or cpu_cores()}"}
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def bench_coverage(args):
    """--config coverage: CoverageStats (CoverageStatisticsCalculator) on yeast 30x
    reads, resident in HBM; a step = one kc_tile_hist pass + D2H of the histograms (1 GPU)."""
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
    # bytes per launch: 12 B per admitted read (global first + span|unique) + the histograms
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
                     "frac": ach / HBM_PEAK_GBS, "traffic": None, "kernel_avg_ms": k_ms,
                     "note": "LDS-bound (difference array + workgroup scan over 4096 positions per tile), not HBM-bound"},
    }), flush=True)


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: run this script under torch.distributed.run as a child (nothing
    here has touched the GPU) and return its exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    if "OMP_NUM_THREADS" not in env:                   # (torch.distributed.run would set 1 for every rank)
        try:
            cores = len(os.sched_getaffinity(0))
        except AttributeError:
            cores = os.cpu_count() or 1
        env["OMP_NUM_THREADS"] = str(max(1, cores // args.gpus))
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--config", default="chr20", choices=["chr20", "yeast", "wgs", "multisample", "coverage"],
                    help="default: chr20 (configs[2]) per GPU at every --gpus N (weak scaling); wgs: configs[3] split "
                         "over the GPUs (strong)")
    ap.add_argument("--no-cold", action="store_true", help="skip the cache-flushed passes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the BAM -> VCF end-to-end run")
    ap.add_argument("--cpu-trunc", type=int, default=2_000_000, help="bp per CPU-baseline piece")
    ap.add_argument("--samples", type=int, default=200)
    ap.add_argument("--contig-first", type=int, default=3, help="multisample: first yeast contig of the shard")
    ap.add_argument("--n-contigs", type=int, default=1, help="multisample: contigs in the shard")
    ap.add_argument("--wgs-shards", type=int, default=0,
                    help="wgs: split the genome over this many shards (default: the world size); with one process, "
                         "--wgs-shard picks the shard this GPU calls (one GPU's part of the 8-GPU split)")
    ap.add_argument("--wgs-shard", type=int, default=-1, help="wgs: the shard to call (default: the rank)")
    args = ap.parse_args()
    if args.config == "multisample" and args.depth == 30.0:
        args.depth = 10.0

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one process per GPU")
        sys.exit(2)
    if args.config == "coverage":
        return bench_coverage(args)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    multi = args.config == "multisample"

    # the CPU baseline runs first, before this process touches the GPU (its oracle pool is child processes); at N > 1
    # on rank 0 only, while the other ranks wait in the process group's rendezvous below
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            t = time.time()
            if multi:
                cpu = cpu_baseline_mvd(args.samples, args.depth)
            elif args.config == "yeast":
                cpu = cpu_baseline(0, 3, args.depth, args.cpu_trunc, 2)
            else:
                cpu = cpu_baseline(1, HUMAN_CHR20, args.depth, args.cpu_trunc, 3)
            log(f"[rank 0] cpu baseline in {time.time() - t:.1f}s: {cpu['value']:.4g} positions/s on {cpu['cores']} cores")
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "error": str(e)}

    dist = None
    backend = os.environ.get("NGSEP_DIST_BACKEND", "nccl")   # gloo: rehearsal of N ranks on fewer GPUs
    if world > 1:
        import torch
        import torch.distributed as tdist
        ndev = torch.cuda.device_count()             # (does not initialise the GPU on this image)
        if backend == "nccl" and ndev < world:
            log(f"bench.py: {world} ranks but {ndev} GPU(s); one process per GPU (NGSEP_DIST_BACKEND=gloo to rehearse)")
            sys.exit(2)
        local_rank = local_rank % max(1, ndev)
        torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend=backend)
        dist = tdist

    import pysynth
    from ngsepcore_amd import GpuPileupSession, default_params
    from ngsepcore_amd.sharding import assign_contigs

    t0 = time.time()
    params = default_params()
    if multi:
        params.multisample = 1
    sessions = []          # (session, synthetic sequences) -- wgs: several device runs of < 2^31 positions
    e2e_src = None
    e2e_indel_src = None
    if multi:
        syn = pysynth.Synth(genome=pysynth.YEAST, depth=args.depth, seed=5, n_samples=args.samples,
                            contig_first=args.contig_first + rank, n_contigs=args.n_contigs)
        names = [n for n, _ in syn.contigs()]
        workload = (f"MultisampleVariantsDetector: {args.samples} synthetic yeast samples at {args.depth:g}x, "
                    f"shard {'+'.join(names)} (one GPU's contig shard of the 8-GPU split)")
        workload_key = f"multisample{args.samples}:{args.depth:g}x:contig{args.contig_first}:v3"
        sources = [syn]
    elif args.config == "yeast":
        sources = [pysynth.Synth(genome=pysynth.YEAST, depth=args.depth, seed=2 + rank)]
        workload = "configs[1]: yeast whole genome (sacCer3 names/lengths, 12,157,105 bp) 30x synthetic 150 bp SE"
        workload_key = f"yeast:{args.depth:g}x:seed{2 + rank}"
    elif args.config == "chr20":
        sources = [pysynth.Synth(genome=pysynth.HUMAN, depth=args.depth, seed=3 + rank, contig_first=HUMAN_CHR20,
                                 n_contigs=1, rng_per_contig=1)]
        workload = "configs[2]: human chr20 (64,444,167 bp) 30x synthetic 150 bp SE"
        workload_key = f"human_chr20:{args.depth:g}x:seed{3 + rank}:v3"
    else:
        # configs[3]: GRCh38 lengths, sequences assigned largest-first to the least-loaded rank; each rank
        # generates and calls only its own (the synthetic sequences are independent: rng_per_contig)
        import ctypes
        lib = pysynth.lib()
        p = pysynth.SynthParams()
        lib.ngs_synth_default(ctypes.byref(p))
        human = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555), ("chr5", 181538259),
                 ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636), ("chr9", 138394717), ("chr10", 133797422),
                 ("chr11", 135086622), ("chr12", 133275309), ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189),
                 ("chr16", 90338345), ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
                 ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]
        nsh = args.wgs_shards if args.wgs_shards > 0 else world
        shard = args.wgs_shard if args.wgs_shard >= 0 else rank
        if world > 1 and nsh != world:
            log("bench.py: --wgs-shards must equal the world size when several ranks run")
            sys.exit(2)
        mine = assign_contigs(human, nsh)[shard]
        idx = [k for k, (n, _) in enumerate(human) if n in mine]
        sources = [("lazy", k) for k in idx]
        workload = (f"configs[3]: human WGS (GRCh38 lengths, 3.10e9 bp) 30x synthetic 150 bp SE, contig-sharded: "
                    f"shard {shard} of {nsh} calls {'+'.join(mine)}")
        workload_key = f"wgs:{args.depth:g}x:shard{shard}of{nsh}"

    # stage: one session per device run (< 2^31 positions each)
    positions = 0
    t_gen = t_stage = 0.0
    reads = read_bases = sites_called = 0
    group, group_len = [], 0
    groups = []
    if sources and isinstance(sources[0], tuple):
        lens = {k: human[k][1] for _, k in sources}
        for _, k in sources:
            if group and group_len + lens[k] > 1_800_000_000:
                groups.append(group)
                group, group_len = [], 0
            group.append(k)
            group_len += lens[k]
        groups.append(group)
    else:
        groups = [[None]]
    for gi, grp in enumerate(groups):
        sess = GpuPileupSession(params, device=local_rank)
        if multi:
            n = max(1, sources[0].params.n_samples)
            sess.set_samples([(f"S{k:03d}", f"S{k:03d}") for k in range(n)])
        for item in grp:
            tg = time.time()
            syn = sources[0] if item is None else pysynth.Synth(genome=pysynth.HUMAN, depth=args.depth, seed=4,
                                                               contig_first=item, n_contigs=1, rng_per_contig=1)
            t_gen += time.time() - tg
            seq_base = len(sess.sequence_names())
            for name, seq in syn.contigs():
                sess.set_reference(name, seq)
            ts = time.time()
            batch = syn.batch()
            if seq_base:
                # the synthetic contig's reads index its own sequence list: shift to the session's indexes
                import ctypes
                import numpy as np
                sid = np.ctypeslib.as_array(batch.seq_id, shape=(batch.n_reads,)) + seq_base
                sid = np.ascontiguousarray(sid, dtype=np.int32)
                batch.seq_id = sid.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            sess.stage(batch)
            t_stage += time.time() - ts
            if item is not None:
                log(f"[rank {rank}] staged {human[item][0]} (device run {gi + 1} of {len(groups)})")
            if args.config == "chr20" and not args.no_e2e:
                # the same reads as a BAM on local disk for the end-to-end run
                tmp = tempfile.mkdtemp(prefix="ngsep_e2e_")
                tw = time.time()
                fa = os.path.join(tmp, "chr20.fa")
                bam = os.path.join(tmp, "chr20.bam")
                pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
                pysynth.lib().ngs_synth_write_bam(syn.h, bam.encode())
                e2e_src = (tmp, fa, bam)
                # the same sequence with indels (rate 1e-4 per position) for the end-to-end run with the indel
                # realigner (its own BAM and FASTA; generated and written untimed; one process only)
                isyn = None if world > 1 else pysynth.Synth(genome=pysynth.HUMAN, depth=args.depth, seed=3 + rank, contig_first=HUMAN_CHR20,
                                     n_contigs=1, rng_per_contig=1, indel_rate=1e-4)
                if isyn is not None:
                    e2e_indel_src = (os.path.join(tmp, "chr20_indels.fa"), os.path.join(tmp, "chr20_indels.bam"))
                    pysynth.lib().ngs_synth_write_fasta(isyn.h, e2e_indel_src[0].encode())
                    pysynth.lib().ngs_synth_write_bam(isyn.h, e2e_indel_src[1].encode())
                    isyn.close()
                log(f"[rank {rank}] wrote the end-to-end BAM ({os.path.getsize(bam) / 1e9:.2f} GB) in {time.time() - tw:.1f}s")
            if multi and rank == 0 and world == 1 and not args.no_e2e:
                # the same population as one BAM per sample on local disk for the end-to-end run
                tmp = tempfile.mkdtemp(prefix="ngsep_e2e_")
                tw = time.time()
                fa = os.path.join(tmp, "shard.fa")
                pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
                bams = syn.write_sample_bams(os.path.join(tmp, "pop"))
                e2e_src = (tmp, fa, bams)
                log(f"[rank 0] wrote {len(bams)} sample BAMs for the end-to-end run in {time.time() - tw:.1f}s")
            if item is not None or len(grp) == 1:
                syn.close()
        ts = time.time()
        sess.stage_finish()
        t_stage += time.time() - ts
        st = sess.stats()
        positions += st.positions_genotyped
        reads += st.alignments_admitted
        read_bases += st.read_bases
        sessions.append(sess)
    log(f"[rank {rank}] generated in {t_gen:.1f}s, staged {reads} reads ({read_bases} read bases) over {positions} "
        f"positions in {t_stage:.1f}s ({len(sessions)} device run(s))")

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        for s in sessions:
            if len(sessions) == 1:
                # the timed loop's own path (two result slots, pinned stores): its buffers reach their size here
                s.submit_staged()
                s.collect_staged()
            else:
                s.run_staged()
    barrier()
    scan_ms, geno_ms = [], []
    t_start = time.perf_counter()
    if len(sessions) == 1:
        # a stream of passes, two in flight: pass k+1's kernels run while pass k's records (multisample: its
        # per-sample calls, gathered into position order) are copied back and collected
        # (ngsep_submit_staged / ngsep_collect_staged); every pass is collected
        sess = sessions[0]
        sess.submit_staged()
        for k in range(args.steps):
            if k + 1 < args.steps:
                sess.submit_staged()
            sess.collect_staged()
            s = sess.stats()
            scan_ms.append(s.scan_ms)
            geno_ms.append(s.genotype_ms)
            sites_called = s.sites_called
    else:
        for k in range(args.steps):
            sites_called = 0
            for sess in sessions:
                sess.run_staged()
                s = sess.stats()
                scan_ms.append(s.scan_ms)
                geno_ms.append(s.genotype_ms)
                sites_called += s.sites_called
    barrier()
    elapsed = time.perf_counter() - t_start
    st = sessions[0].stats()
    log(f"[rank {rank}] tile {st.tile_positions} positions (max {st.tile_rows_max} rows), pile {st.pile_bytes} B, "
        f"{st.candidates} candidates, {st.hard_sites} needed the exact tally + posterior, {sites_called} calls")
    cold = cold_passes(sessions[0]) if world == 1 and not args.no_cold and len(sessions) == 1 else None
    stats_all = [s.stats() for s in sessions]
    pile_bytes = sum(x.pile_bytes for x in stats_all)
    tile = st.tile_positions
    # bytes the scan kernel moves per launch.  KL: the read-group units (1 B per read base, zero padded to the
    # group's longest read in 8-B units; stats.pile_bytes), 8-B entry headers, 16 B per 64-read group, the
    # reference codes (1 B per global position, halos included) and the two block tables (8 B per 256
    # positions).  The multisample scan (KLM + KQN) reads the population read-group layout the same way (units,
    # headers, groups) plus its tile's reference codes once per four samples, and sets / scans the open-position
    # bits (1 bit per global position)
    if multi:
        kt_bytes = sum(x.pile_bytes + 8 * x.alignments_admitted + 16 * ((x.alignments_admitted + 63) // 64) +
                       x.global_positions * ((args.samples + 3) // 4) + x.global_positions // 4 for x in stats_all)
    else:
        kt_bytes = sum(x.pile_bytes + 8 * x.alignments_admitted + 16 * ((x.alignments_admitted + 63) // 64) +
                       x.global_positions + x.global_positions // 32 for x in stats_all)
    layout_ms = sum(x.layout_ms for x in stats_all)
    upload_ms = sum(x.upload_ms for x in stats_all)
    for s in sessions:
        s.release_staged()
        s.close()

    e2e = None
    if e2e_src is not None:
        try:
            e2e = (end_to_end_population if multi else end_to_end)(e2e_src[1], e2e_src[2], local_rank)
            log(f"[rank {rank}] end-to-end BAM -> VCF: {e2e['wall_s']:.2f}s, {e2e['value']:.4g} positions/s")
            if e2e_indel_src is not None:
                r = end_to_end(e2e_indel_src[0], e2e_indel_src[1], local_rank)
                r["note"] += "; synthetic indels at rate 1e-4 per position (the indel realigner's regions replayed)"
                e2e["indels"] = r
                log(f"[rank 0] end-to-end with indels: {r['wall_s']:.2f}s, {r['value']:.4g} positions/s, "
                    f"{r['realign_regions']} realigner regions replayed in {r['realign_replay_ms']:.1f} ms")
        except Exception as e:
            e2e = {"value": None, "error": str(e)}
        finally:
            shutil.rmtree(e2e_src[0], ignore_errors=True)
    elif args.config == "wgs" and rank == 0 and world == 1 and not args.no_e2e:
        # configs[3] shard end to end: each of the shard's sequences as a BAM on local disk (written untimed), then
        # BAM -> VCF through ngsep_call_bam; wall times and positions summed over the shard
        try:
            tot_wall = tot_pos = tot_bytes = tot_rec = 0
            for _, k in sources:
                tmp = tempfile.mkdtemp(prefix="ngsep_e2e_")
                try:
                    syn = pysynth.Synth(genome=pysynth.HUMAN, depth=args.depth, seed=4, contig_first=k, n_contigs=1,
                                        rng_per_contig=1)
                    fa, bam = os.path.join(tmp, "c.fa"), os.path.join(tmp, "c.bam")
                    pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
                    pysynth.lib().ngs_synth_write_bam(syn.h, bam.encode())
                    syn.close()
                    r = end_to_end(fa, bam, local_rank)
                    log(f"[rank 0] end-to-end {human[k][0]}: {r['wall_s']:.2f}s, {r['value']:.4g} positions/s")
                    tot_wall += r["wall_s"]
                    tot_pos += r["positions"]
                    tot_bytes += r["bam_bytes"]
                    tot_rec += r["vcf_records"]
                finally:
                    shutil.rmtree(tmp, ignore_errors=True)
            e2e = {"wall_s": tot_wall, "positions": tot_pos, "value": tot_pos / tot_wall, "unit": "positions/s",
                   "vcf_records": tot_rec, "bam_bytes": tot_bytes,
                   "note": "ngsep_call_bam per sequence of the shard: BAM on disk -> VCF on disk incl. FASTA load, "
                           f"summed; host threads {os.environ.get('NGSEP_THREADS') or cpu_cores()}"}
        except Exception as e:
            e2e = {"value": None, "error": str(e)}

    sharded = None
    if dist is not None and e2e is not None and args.config == "chr20":
        # every rank its own BAM -> VCF (the N = 1 leg per GPU): the slowest rank's wall, positions summed
        import torch
        ok = e2e.get("value") is not None
        t = torch.tensor([e2e.get("wall_s", 0.0) if ok else 0.0, float(e2e.get("positions", 0) if ok else 0), 0.0 if ok else 1.0],
                         dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        mx = t[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t[1:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        if rank == 0:
            if float(sm[1]) > 0:
                e2e = {"value": None, "error": f"{int(sm[1])} rank(s) failed the end-to-end leg", "rank0": e2e}
            else:
                e2e = dict(e2e, wall_s=float(mx[0]), positions=int(sm[0]), value=float(sm[0]) / float(mx[0]),
                           rank0_wall_s=e2e["wall_s"],
                           note=e2e["note"] + f"; every rank its own chr20 BAM (seed 3 + rank): the slowest rank's wall, "
                                              f"positions summed over {world} ranks")
    if dist is not None and not args.no_e2e and args.config in ("wgs", "chr20"):
        try:
            sharded = sharded_end_to_end(args, dist, rank, local_rank, backend)
            if rank == 0:
                log(f"[rank 0] sharded end-to-end over {world} ranks: {sharded['wall_s']:.2f}s, {sharded['windows']} windows")
        except Exception as ex:
            sharded = {"value": None, "error": str(ex)}
        if args.config == "wgs":
            e2e, sharded = sharded, None
    if dist is not None:
        import torch
        t = torch.tensor([elapsed, float(positions)], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
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
        k_avg_ms = sum(scan_ms) / len(scan_ms) * (len(sessions) if len(sessions) > 1 else 1)
        post_avg_ms = (sum(geno_ms) / len(geno_ms)) if max(geno_ms, default=0) > 0 else None
        # SURVEY.md 8(d)'s algorithmic bytes (1 B per read base + 1 B reference per genotyped position + 16 B per
        # read) per launch: `achieved` for the single-sample scan KL, which reads exactly that input
        alg_bytes = read_bases + positions + 16 * reads
        # (the multisample scan KLM reads the same input: every sample's read-group units)
        achieved = alg_bytes / (k_avg_ms * 1e-3) / 1e9 if k_avg_ms > 0 else None
        traffic = load_traffic(workload_key)
        scan_kernel = "k_scan_pop+k_queue_need" if multi else f"k_read_scan<{tile}>"
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "positions/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / steps,
            "higher_is_better": True,
            "scaling": "strong" if args.config == "wgs" else "weak",
            "vs_baseline": None,
            "dtype": "u8,f64",
            "data": ("synthetic (seeded generator, SURVEY.md 8(d)); " +
                     ("the host packer's population read-group layout (1 B per read base, one stream per sample) "
                      "resident in HBM; the step scans it" if multi else
                      "the host packer's read-group layout (1 B per read base) resident in HBM; the step scans it")),
            "config": {
                "workload": workload,
                "positions_per_gpu": positions,
                "reads_per_gpu": int(reads),
                "read_bases_per_gpu": int(read_bases),
                "sites_called_per_gpu": int(sites_called),
                "candidates_per_gpu": int(st.candidates),
                "exact_sites_per_gpu": int(st.hard_sites),
                "exact_bound_columns_per_gpu": int(st.exact_bound_passes),
                "pile_bytes_per_gpu": int(pile_bytes),
                "tile_positions": int(tile),
                "device_runs_per_gpu": len(sessions),
                "host_layout_ms": layout_ms,
                "h2d_upload_ms": upload_ms,
                "parallelism": (f"dp{world} (contig split of the genome over the GPUs, no collective)" if args.config == "wgs"
                                else f"dp{world} (independent genomic windows per GPU, no collective)"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": scan_kernel,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": traffic,
                "bytes_per_launch": alg_bytes,
                "bytes_moved_per_launch": kt_bytes,
                "kernel_avg_ms": k_avg_ms,
                "traffic_rate_GBs": (traffic / (k_avg_ms * 1e-3) / 1e9) if traffic and k_avg_ms > 0 else None,
                "alg_bytes_per_launch": alg_bytes,
                "alg_equiv_GBs": alg_bytes / (k_avg_ms * 1e-3) / 1e9 if k_avg_ms > 0 else None,
                "cold": cold,
                # KP is timed only with NGSEP_TIME_POSTERIOR=1 (its event costs a few us of pipeline gap)
                "posterior_kernel_avg_ms": post_avg_ms,
            },
        }
        from ngsepcore_amd import _lib as nlib
        if nlib.LIB_PATH != nlib.DEFAULT_LIB_PATH:      # an A/B tuning build (NGSEP_LIB_PATH): named in the line
            line["config"]["lib_path"] = nlib.LIB_PATH
        if multi:
            line["config"]["samples"] = args.samples
            line["config"]["sample_calls_per_step"] = int(sites_called) * args.samples
        if e2e is not None:
            line["end_to_end"] = e2e
        if sharded is not None:
            line["sharded_end_to_end"] = sharded
        if cpu is not None:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
