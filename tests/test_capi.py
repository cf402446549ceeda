"""The C-ABI library loads and exports every entry point include/ngsep_gpu.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

from ngsepcore_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ngsep_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ngsep_[a-z_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding covers every one of them
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_abi_version_and_defaults():
    lib = _lib.load()
    assert lib.ngsep_abi_version() == 12
    p = _lib.NgsepParams()
    lib.ngsep_params_default(ctypes.byref(p))
    # DEF_* constants: SingleSampleVariantsDetector.java:65-78, CountsHelper.java:42-48
    assert (p.min_mq, p.max_alns_per_start, p.max_base_qs, p.min_quality, p.ploidy) == (20, 5, 30, 40, 2)
    assert p.het_rate == 0.001 and p.sample_id == b"Sample" and p.query_last == 1000000000


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_lib.NgsepSiteOut) == 152
    assert ctypes.sizeof(_lib.NgsepReadBatch) == 8 + 12 * 8


def test_unsupported_inputs_fail_loudly():
    from ngsepcore_amd import GpuPileupSession, NgsepError
    p = _lib.NgsepParams()
    _lib.load().ngsep_params_default(ctypes.byref(p))
    p.ploidy = 129          # the pool algorithm's hypotheses table holds ploidy <= 128
    with pytest.raises(NgsepError) as e:
        GpuPileupSession(p)
    assert e.value.code == _lib.NGSEP_E_UNSUPPORTED


@pytest.mark.skipif(_lib.load().ngsep_device_count() > 0, reason="checks the no-GPU failure mode")
def test_no_device_fails_loudly(tmp_path):
    """Without an MI355X the product refuses to run (there is no CPU fallback)."""
    import pysynth
    from ngsepcore_amd import GpuPileupSession, NgsepError
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=5000, depth=5, seed=1)
    with GpuPileupSession() as s:
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        with pytest.raises(NgsepError) as e:
            s.processAlignments(syn.batch())
            s.notifyEndOfAlignments()
        assert e.value.code == _lib.NGSEP_E_DEVICE


def test_known_strs_argument_checks(tmp_path):
    """ngsep_set_known_strs (ABI 7): needs the reference first, belongs to the variant detectors only, reads
    its file; lines the reference's loader skips (SimpleGenomicRegionFileHandler.java:57-80) are skipped here too."""
    from ngsepcore_amd import GpuPileupSession, NgsepError, default_params
    path = os.path.join(str(tmp_path), "strs.txt")
    with open(path, "w") as f:
        f.write("c1\t10\t20\nc1 30 40\nnope\t1\t2\nc1\tx\t3\nc1\t5\n\n")
    with GpuPileupSession() as s:
        with pytest.raises(NgsepError) as e:
            s.set_known_strs(path)
        assert e.value.code == _lib.NGSEP_E_INVALID
        s.set_reference("c1", b"ACGT" * 100)
        s.set_known_strs(path)
        s.set_known_strs(None)
        with pytest.raises(NgsepError) as e:
            s.set_known_strs(os.path.join(str(tmp_path), "missing.txt"))
        assert e.value.code == _lib.NGSEP_E_IO
    p = default_params()
    p.multisample = 1                       # MultisampleVariantsDetector -knownSTRs (:439-446): accepted (ABI 8)
    with GpuPileupSession(p) as s:
        s.set_reference("c1", b"ACGT" * 100)
        s.set_known_strs(path)
    p = default_params()
    p.coverage_stats = 1
    with GpuPileupSession(p) as s:
        s.set_reference("c1", b"ACGT" * 100)
        with pytest.raises(NgsepError) as e:
            s.set_known_strs(path)
        assert e.value.code == _lib.NGSEP_E_INVALID
