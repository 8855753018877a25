"""shrewd_amd -- MI355X-native fault-injection campaign engine for SHREWD/gem5.

The hot path (RV64 AtomicSimpleCPU SE-mode trials, one per GPU lane) runs in
hand-written HIP kernels behind the C ABI in include/fi_engine.h; this package
is the host-side mirror of the gem5 FaultCampaign SimObject interface.
"""
from .fi import (CLASS_NAMES, CRASH_NAMES, END_NAMES, ESCAPE_NAMES, HANG_NAMES, FaultCampaign, Engine, EngineError,
                 HIST_DT, OUTCOME_DT, SITE_DT, allreduce_histogram, build_library, library_path, shard_range,
                 structures_mask)

__all__ = ["FaultCampaign", "Engine", "EngineError", "OUTCOME_DT", "SITE_DT", "HIST_DT", "CLASS_NAMES",
           "CRASH_NAMES", "ESCAPE_NAMES", "HANG_NAMES", "END_NAMES", "allreduce_histogram", "build_library",
           "library_path", "shard_range", "structures_mask"]
