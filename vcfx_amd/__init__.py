"""vcfx_amd -- MI355X-native engine for the VCFX per-record hot path.

Product layout:
  build/libvcfx_gpu.so     HIP/CDNA4 record engine behind the C ABI of include/vcfx_gpu.h
  build/libvcfx_tools.so   the VCFX_<tool> drop-ins (same CLI contract as the reference)
  build/src/VCFX_<t>/VCFX_<t>  executables
Python: vcfx_amd.engine (ctypes view of the C ABI), vcfx_amd.tools (in-process tool runs).
There is no CPU fallback: every compute call fails loudly without a gfx950 device.
"""
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "build")
GPU_LIB = os.environ.get("VCFXG_GPU_LIB") or os.path.join(BUILD, "libvcfx_gpu.so")  # env: experiment builds
TOOLS_LIB = os.path.join(BUILD, "libvcfx_tools.so")
SYNTH_LIB = os.path.join(BUILD, "libvcfx_synth.so")
TOOLS = ("VCFX_allele_freq_calc", "VCFX_record_filter", "VCFX_genotype_query", "VCFX_ld_calculator",
         "VCFX_variant_counter")


def tool_binary(tool):
    return os.path.join(BUILD, "src", tool, tool)
