// gen_tables.cpp -- writes errmod_tables.bin (the constant cal_coef tables of
// errmod_init(1.0-0.83), pop_utils.cpp:203-266) beside libpopbam_gpu.so at build time, so a
// context reads them instead of recomputing them (pbg_host.h load_errmod_tables).
#include <cstdio>

#include "pbg_host.h"

int main(int argc, char **argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: gen_tables <out.bin>\n");
        return 2;
    }
    if (!pbg::write_errmod_tables(argv[1])) {
        std::fprintf(stderr, "gen_tables: cannot write %s\n", argv[1]);
        return 1;
    }
    return 0;
}
