// pipe_main.cpp -- the vcfx_pipe executable (tool_pipe.cpp, include/vcfx_tools.h).
#include <stdio.h>
#include <unistd.h>

#include "hostio.h"
#include "tools.h"

int main(int argc, char **argv) {
    vcfxh::g_process_exit_fast = true;
    const int rc = vcfx_pipe_main(argc, argv, 0, 1, 2);
    vcfxh::phase("pipe done");
    // every byte is written; end without the HIP runtime's teardown (binary_main.cpp)
    vcfxh::gpu_join();
    fflush(nullptr);
    _exit(rc);
}
