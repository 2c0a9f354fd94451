// Test driver for INTEGRATION.md (test infrastructure; nothing in the product links it).
//
// The document's c++ blocks -- the pileup callback pbg_collect, the streamed run that replaces
// main_<cmd>'s window loop and main_nucdiv_gpu / main_sfs_gpu / main_ld_gpu -- are extracted
// verbatim (oracle/extract_integration.py) and compiled here against the reference's own
// headers, linked with the reference's own objects (POPBAM 0.3 built by this directory's
// Makefile from /root/reference; popbam.o with its main renamed) and libpopbam_gpu.so.  main
// dispatches like popbam.cpp:53-77.  tests/test_integration.py runs the binary on the golden
// BAMs and compares its stdout with the reference's.
//
// nucdivData keeps min_sites private (pop_nucdiv.h:53); the document has the maintainer add a
// friend declaration.  Here the reference's headers are read with `private` defined as
// `public` instead (after every standard header they include, so only their own classes see
// it): same layout, same objects, no edited reference file.
#include <algorithm>
#include <cassert>
#include <cerrno>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <limits>
#include <map>
#include <new>
#include <sstream>
#include <string>
#include <vector>
#include <sys/stat.h>

#define private public
#include "pop_nucdiv.h"
#include "pop_sfs.h"
#include "pop_ld.h"
#undef private

#include "integration_blocks.inc"

int main(int argc, char *argv[])
{
    if (argc < 2) {
        std::cerr << "usage: popbam_integ nucdiv|sfs|ld [options] <in.bam> <region>" << std::endl;
        return 1;
    }
    if (!strcmp(argv[1], "nucdiv")) return main_nucdiv_gpu(argc - 1, argv + 1);
    if (!strcmp(argv[1], "sfs")) return main_sfs_gpu(argc - 1, argv + 1);
    if (!strcmp(argv[1], "ld")) return main_ld_gpu(argc - 1, argv + 1);
    std::cerr << "Error: unrecognized command: " << argv[1] << std::endl;
    return 1;
}
