"""Host-code sanitizer runs of the whole pipeline on a GPU box.

The ngsep-amd CLI is built three ways from the same sources (ngsepcore_amd/csrc/Makefile):
  lib/       release
  lib_asan/  SAN=address,undefined  (host code instrumented with -Xarch_host; the CLI links the clang runtime)
  lib_tsan/  SAN=thread
Each variant runs SingleSampleVariantsDetector on an indel-bearing BAM (decoder, prefetch, window worker,
device-init threads, the realigner's host replay, streamed windows), with -knownSTRs, MultisampleVariantsDetector
on 12 sample BAMs, CoverageStats and RelativeAlleleCounts.  The VCFs must equal the oracle's, the reports the
release build's, and the sanitizers must report nothing (exit code != 0 on any report).

This process never touches the GPU itself: it generates data (tools/synth), runs the oracle (CPU) and starts the
CLIs as child processes.  Usage: python tools/san_cli.py OUTDIR [variant ...]
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ngsep_oracle  # noqa: E402
import pysynth  # noqa: E402

ENV = {
    "asan": {"ASAN_OPTIONS": "detect_leaks=0:protect_shadow_gap=0:abort_on_error=0:exitcode=86",
             "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1:exitcode=87"},
    "tsan": {"TSAN_OPTIONS": "exitcode=88:report_signal_unsafe=0:second_deadlock_stack=1:ignore_noninstrumented_modules=1"},
    "release": {},
}


def records(path):
    if not os.path.exists(path):
        return None
    return [l for l in open(path) if not l.startswith("#")]


def run(variant, args, log):
    cli = os.path.join(ROOT, "ngsepcore_amd", "lib" if variant == "release" else f"lib_{variant}", "ngsep-amd")
    env = dict(os.environ)
    env.update(ENV[variant])
    t0 = time.time()
    with open(log, "w") as f:
        rc = subprocess.run(["timeout", "-k", "10", "300", cli] + args, stdout=f, stderr=subprocess.STDOUT, env=env).returncode
    txt = open(log).read()
    bad = rc != 0 or "ERROR: AddressSanitizer" in txt or "runtime error:" in txt or "WARNING: ThreadSanitizer" in txt
    print(f"[{variant}] {' '.join(args[:1])} rc={rc} {time.time() - t0:.1f}s {'SANITIZER/FAIL' if bad else 'clean'}", flush=True)
    if bad:
        print(txt[-4000:], flush=True)
    return not bad


def main():
    out = os.path.abspath(sys.argv[1])
    variants = sys.argv[2:] or ["release", "asan", "tsan"]
    os.makedirs(out, exist_ok=True)
    ok = True
    # single sample with indels (realigner regions on the host, streamed windows of 60 kb)
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=20, seed=36, indel_rate=3e-4, snv_rate=3e-3)
    fa, sam, bam = syn.write(os.path.join(out, "ind"))
    syn.close()
    ngsep_oracle.run_ssvd(fa, sam, os.path.join(out, "oracle.vcf"), call_embedded=1)
    # population of 12 sample BAMs
    pop = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=60000, depth=10, seed=5, n_samples=12, snv_rate=2e-3)
    pfa, psam, _ = pop.write(os.path.join(out, "pop"))
    pbams = pop.write_sample_bams(os.path.join(out, "pop"))
    pop.close()
    ngsep_oracle.run_mvd(pfa, psam, os.path.join(out, "oracle_mvd.vcf"), 0.0)
    reports = {}
    for v in variants:
        ok &= run(v, ["SingleSampleVariantsDetector", "-i", bam, "-r", fa, "-o", os.path.join(out, f"ss_{v}"), "-embeddedSNVs"],
                  os.path.join(out, f"ss_{v}.log"))
        same = records(os.path.join(out, f"ss_{v}.vcf")) == records(os.path.join(out, "oracle.vcf"))
        print(f"[{v}] single-sample VCF == oracle: {same}", flush=True)
        ok &= same
        ok &= run(v, ["MultisampleVariantsDetector", "-r", pfa, "-o", os.path.join(out, f"mvd_{v}.vcf")] + pbams,
                  os.path.join(out, f"mvd_{v}.log"))
        same = records(os.path.join(out, f"mvd_{v}.vcf")) == records(os.path.join(out, "oracle_mvd.vcf"))
        print(f"[{v}] population VCF == oracle: {same}", flush=True)
        ok &= same
        ok &= run(v, ["CoverageStats", "-i", bam, "-r", fa, "-o", os.path.join(out, f"cov_{v}.txt")], os.path.join(out, f"cov_{v}.log"))
        ok &= run(v, ["RelativeAlleleCounts", "-i", bam, "-r", fa, "-o", os.path.join(out, f"rac_{v}.txt")], os.path.join(out, f"rac_{v}.log"))
        reports[v] = tuple(open(p).read() if os.path.exists(p) else None
                           for p in (os.path.join(out, f"cov_{v}.txt"), os.path.join(out, f"rac_{v}.txt")))
    if "release" in reports:
        for v, r in reports.items():
            same = r == reports["release"]
            print(f"[{v}] coverage / RAC reports == release: {same}", flush=True)
            ok &= same
    for f in glob.glob(os.path.join(out, "*.bam")) + glob.glob(os.path.join(out, "*.sam")):
        os.remove(f)
    print("SANITIZER RUNS", "PASSED" if ok else "FAILED", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
