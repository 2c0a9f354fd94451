// pbg_key.h -- call_base's per-read part (popbam.cpp:266-287), shared by the host side of the
// pileup callback (feeder.cpp) and the synthetic generator kernels (call_kernel.hip).
#pragma once
#include <stdint.h>

#ifndef PBG_HD
#define PBG_HD
#endif

namespace pbg {

// A raw read word (bits 0-7 bam1_qual()[qpos], 8-15 core.qual, 16-19 nt16 base, bit 20
// bam1_strand) -> the u16 key qq<<5 | strand<<4 | base, or 0 when call_base skips the read:
// baseQ (after the Illumina 1.3+ offset, floor 0) < min_baseQ, mapQ < min_mapQ, or a base
// that bam_nt16_nt4_table does not map to A/C/G/T.  qq = clamp(min(baseQ, mapQ), 4, 63), so a
// key is never 0.  mapq (out) = core.qual, whose square call_base adds to rmsq.
PBG_HD inline uint32_t read_to_key(uint32_t r, uint32_t min_baseQ, uint32_t min_mapQ, bool illumina) {
    const uint32_t raw = r & 0xffu;
    const uint32_t bq = illumina ? (raw > 31u ? raw - 31u : 0u) : raw;
    const uint32_t mq = (r >> 8) & 0xffu;
    const uint32_t nt = (r >> 16) & 0xfu;
    if (bq < min_baseQ || mq < min_mapQ) return 0u;
    if (nt != 1u && nt != 2u && nt != 4u && nt != 8u) return 0u;
    const uint32_t b = nt == 1u ? 0u : nt == 2u ? 1u : nt == 4u ? 2u : 3u;
    uint32_t qq = bq < mq ? bq : mq;
    qq = qq < 4u ? 4u : (qq > 63u ? 63u : qq);
    return (qq << 5) | (((r >> 20) & 1u) << 4) | b;
}

}  // namespace pbg
