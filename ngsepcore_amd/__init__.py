"""ngsepcore_amd -- MI355X-native drop-in for NGSEP's SNV pileup-calling path.

The compute path is libngsep_amd.so (HIP kernels for gfx950 behind the C ABI in
include/ngsep_gpu.h); this package is the host-side mirror of the reference interface.
"""
from ._lib import LIB_PATH, NgsepError, load  # noqa: F401
from .discovery import (CalledSite, CoverageStatisticsCalculator, GpuPileupSession, MultisampleVariantsDetector, PopulationSite,  # noqa: F401
                        RelativeAlleleCountsCalculator, SingleSampleVariantsDetector, default_params)

__all__ = ["GpuPileupSession", "CoverageStatisticsCalculator", "RelativeAlleleCountsCalculator", "SingleSampleVariantsDetector", "MultisampleVariantsDetector", "PopulationSite", "CalledSite", "NgsepError", "default_params",
           "load", "LIB_PATH"]
