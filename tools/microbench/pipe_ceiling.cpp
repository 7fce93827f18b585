// vcfx_pipe_ceiling -- the stdin-pipe ceiling of the device-only AF path on this host: the
// drop-in's own reader (vcfxh::Input::read_fd with host_copy = false: F_SETPIPE_SZ, the head
// prefaulted on a helper core, catch_up, the pinned 16 x 1 MiB staging ring) with the device
// stage stubbed (tests/shard_tsan_stub.cpp built with -DVCFX_STUB_DISCARD: vcfxg_ingest takes
// each chunk and keeps nothing, no HIP runtime).  bench.py's e2e leg times
// `cat F | vcfx_pipe_ceiling` beside `cat F | VCFX_allele_freq_calc -q`: what the tool adds on
// top of its own reader is the device (HIP start, DMA, kernels, rows).
#include "hostio.h"

int main() {
    vcfxh::Input in;
    in.read_fd(0, false);
    return in.read_errno ? 1 : 0;
}
