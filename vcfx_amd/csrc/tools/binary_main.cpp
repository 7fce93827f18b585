// tool_binary_main.cpp -- the VCFX_<tool> executable: main() of the drop-in binary.
// VCFX_TOOL_NAME is set per binary at compile time.
#include "tools.h"

int main(int argc, char **argv) { return vcfx_tool_main(VCFX_TOOL_NAME, argc, argv, 0, 1, 2); }
