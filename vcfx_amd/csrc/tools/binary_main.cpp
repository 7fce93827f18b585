// tool_binary_main.cpp -- the VCFX_<tool> executable: main() of the drop-in binary.
// VCFX_TOOL_NAME is set per binary at compile time.
#include <stdio.h>
#include <unistd.h>

#include "hostio.h"
#include "tools.h"

int main(int argc, char **argv) {
    vcfxh::g_process_exit_fast = true;
    int rc = vcfx_tool_main(VCFX_TOOL_NAME, argc, argv, 0, 1, 2);
    vcfxh::phase("tool done");
    // every byte is written (the tools' writers flush on return); end without running the
    // HIP runtime's teardown and unmapping the input (~0.1 s at 4 GB; the kernel releases
    // the device and the mappings at exit either way)
    vcfxh::gpu_join();
    fflush(nullptr);
    _exit(rc);
}
