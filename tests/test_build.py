"""CPU checks of the product build: the C-ABI library loads and exports every symbol
include/vcfx_gpu.h declares; tool entry points exist; no GPU is needed for these."""
import ctypes
import os
import re

import pytest

from vcfx_amd import BUILD, GPU_LIB, TOOLS, TOOLS_LIB, tool_binary
from vcfx_amd import engine

HDR = os.path.join(os.path.dirname(BUILD), "include", "vcfx_gpu.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(vcfxg_[a-z0-9_]+)\s*\(", txt)))


def test_gpu_lib_exports_header_symbols():
    lib = ctypes.CDLL(GPU_LIB)
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    assert set(declared_symbols()) == set(engine.SIGNATURES)


def test_open_without_gpu_fails_loudly():
    n = ctypes.c_int(-1)
    engine.lib().vcfxg_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(engine.EngineError):
        engine.Engine(0)


def test_tools_lib_exports():
    lib = ctypes.CDLL(TOOLS_LIB)
    txt = open(os.path.join(os.path.dirname(BUILD), "include", "vcfx_tools.h")).read()
    syms = sorted(set(re.findall(r"\b(vcfx_(?:tool|pipeline|shard)_[a-z0-9_]+)\s*\(", txt)))
    assert len(syms) == 15, syms  # main, 11 tools, the fused pipeline, the sharded main and its plan
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


@pytest.mark.parametrize("tool", ["VCFX_allele_freq_calc", "VCFX_genotype_query", "VCFX_record_filter", "VCFX_variant_counter", "VCFX_ld_calculator",
                                  "VCFX_nonref_filter", "VCFX_hwe_tester", "VCFX_dosage_calculator", "VCFX_missing_detector",
                                  "VCFX_allele_counter", "VCFX_haplotype_phaser"])
def test_binaries_present(tool):
    assert os.access(tool_binary(tool), os.X_OK)


def test_shard_cuts_abi_matches_rule():
    """vcfxg_shard_cuts (C ABI, no device) against the numpy restatement of the reference's
    split (VCFX_allele_counter.cpp:889-901) on ragged inputs, every world size 1..9"""
    import numpy as np
    from vcfx_amd import shard
    rng = np.random.default_rng(7)
    for trial in range(40):
        n = int(rng.integers(0, 5000))
        arr = rng.integers(32, 127, n).astype(np.uint8)
        arr[rng.random(n) < rng.choice([0.0, 0.001, 0.05, 0.5])] = 10
        buf = arr.tobytes()
        lo = int(rng.integers(0, n + 1))
        for world in range(1, 10):
            assert engine.shard_cuts(buf, lo, world) == shard.record_cuts_py(buf, lo, world), (trial, world)
