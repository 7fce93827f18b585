// tool_binary_main.cpp -- the VCFX_<tool> executable: main() of the drop-in binary.
// VCFX_TOOL_NAME is set per binary at compile time.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "hostio.h"
#include "tools.h"

// VCFX_NGPU: ranks of the in-process multi-GPU run (a count, or "all" = every device)
static int ngpu_env() {
    const char *e = getenv("VCFX_NGPU");
    if (!e || !*e) return 1;
    if (!strcmp(e, "all")) {
        int n = 0;
        return vcfxg_device_count(&n) == VCFXG_OK && n > 0 ? n : 1;
    }
    const int n = atoi(e);
    return n > 1 ? n : 1;
}

int main(int argc, char **argv) {
    vcfxh::g_process_exit_fast = true;
    const int ngpu = ngpu_env();
    int rc = ngpu > 1 ? vcfx_tool_main_sharded(VCFX_TOOL_NAME, argc, argv, 0, 1, 2, ngpu)
                      : vcfx_tool_main(VCFX_TOOL_NAME, argc, argv, 0, 1, 2);
    vcfxh::phase("tool done");
    // every byte is written (the tools' writers flush on return); end without running the
    // HIP runtime's teardown and unmapping the input (~0.1 s at 4 GB; the kernel releases
    // the device and the mappings at exit either way)
    vcfxh::gpu_join();
    fflush(nullptr);
    _exit(rc);
}
