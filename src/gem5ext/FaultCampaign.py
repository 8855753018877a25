# FaultCampaign SimObject -- drop-in campaign front end for gem5.
#
# Declared the way gem5 declares SimObjects (type / cxx_header / cxx_class /
# Param.*; pattern of src/cpu/o3/BaseO3CPU.py:64-72) with Python-callable
# methods exported through cxx_exports (src/cpu/BaseCPU.py:68-77, the same
# mechanism SHREWD uses for setEnableShrewd).  Built into gem5 out of tree with
#   scons build/RISCV/gem5.opt EXTRAS=/path/to/this/repo/src/gem5ext
# (SConstruct:882-897).  The C++ side (fault_campaign.{hh,cc}) drives the
# MI355X engine through the C ABI include/fi_engine.h via src/campaign/.
from m5.params import *
from m5.SimObject import PyBindMethod, SimObject


class FaultCampaign(SimObject):
    type = "FaultCampaign"
    cxx_header = "gem5ext/fault_campaign.hh"
    cxx_class = "gem5::FaultCampaign"
    cxx_exports = [
        PyBindMethod("run"),
        PyBindMethod("summaryJson"),
        PyBindMethod("setProtectMask"),
        PyBindMethod("setProtectOpClasses"),
        PyBindMethod("trialsRun"),
        PyBindMethod("histogram"),
    ]

    workload = Param.String("RV64 static ELF run in SE mode")
    cmd = VectorParam.String([], "argv of the workload (cmd[0] defaults to workload)")
    checkpoint = Param.String(
        "", "gem5 SE checkpoint directory the trials start from (m5.cpt + memory store); "
        "empty: process start")
    env = VectorParam.String([], "environment of the workload")
    executable = Param.String(
        "", "Process.executable: readlinkat('/proc/self/exe') answers its realpath (empty: the workload path)")
    input = Param.String(
        "cin", "Process.input: 'cin' = the host's stdin (reads of fd 0 end the trial as escape/host); "
        "else a file fd 0 reads, deterministically per trial")
    trials = Param.UInt64(1000, "number of fault-injection trials")
    first_trial = Param.UInt64(0, "first trial id (sites are keyed by (seed, trial id))")
    seed = Param.UInt64(0x5EED0001, "campaign seed")
    structures = VectorParam.String(
        ["int_reg"], "fault targets: int_reg, pc, mem, result, xN or ABI register names")
    bits = Param.String(
        "0-63", "eligible lowest flipped bit positions: ranges / positions ('0-31,63') or a mask")
    burst = Param.UInt32(1, "adjacent bits flipped per fault (1..64)")
    protect_mask = Param.UInt64(
        0, "selective replication: protected x0..x31 (bits 0-31) and pc (bit 32)")
    protect_opclasses = VectorParam.String(
        [], "SHREWD replication: gem5 OpClass names whose instructions get a shadow "
        "execution (IntAlu, IntMult, IntDiv, Float*); a result fault on one is detected")
    shadow_fu_model = Param.Bool(
        False, "SHREWD FU contention: a protected instruction is replicated only if its "
        "shadow finds a free functional unit in an O3 issue model of the golden run "
        "(FUPool::getUnit / InstructionQueue::requestShadow)")
    priority_to_shadow = Param.Bool(
        False, "shadows claim units before younger primaries (BaseO3CPU.priorityToShadow)")
    issue_width = Param.UInt32(8, "issue model: instructions issued per cycle (BaseO3CPU.issueWidth)")
    load_latency = Param.UInt32(2, "issue model: cycles from a load's issue to its value")
    cpu_type = Param.String(
        "atomic", "time coordinate of the fault sites: 'atomic' (a committed-instruction count, "
        "AtomicSimpleCPU) or 'timing' (a tick of a TimingSimpleCPU run on the NoCache + "
        "SingleChannelDDR3_1600 board of the SE run script)")
    num_gpus = Param.UInt32(1, "MI355X devices used by this process")
    first_gpu = Param.UInt32(0, "first HIP device ordinal")
    max_insts_factor = Param.Float(
        2.0, "hang cap: golden committed instructions x factor + 1000")
    private_pages = Param.UInt32(16, "copy-on-write guest pages per trial")
    output = Param.String("", "prefix for outcome/histogram files (empty: none)")
