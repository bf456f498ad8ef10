/* zpaq_standin.h -- a STAND-IN for the reference's boundary chunker, for
 * timing only.  Not the crate's boundaries.
 *
 * The reference cuts every file with cdchunking 0.2.1's
 * Chunker::new(ZPAQ::new(13)).max_size(32768) (/root/reference/src/index.rs:
 * 40-41, 622-625; Cargo.lock:42-45), whose source is not in this image and
 * whose recurrence could not be pinned to the reference's known-answer test
 * (DESIGN.md section 2.3).  This is zpaq's fragmenter in the survey's form
 * (SURVEY.md section 0.3, Appendix A): per byte, one order-1 prediction-table
 * lookup, a compare, an add and a 32-bit multiply,
 *     h = (h + c + 1) * (c == o1[c1] ? 314159265 : 271828182),
 *     o1[c1] = c, c1 = c,
 * a boundary after the byte when h < 2^(32 - bits), and a forced one at
 * max_size, with the state reset at every boundary (a chunk's state starts
 * fresh, which read_block relies on, src/sync/fs.rs:26-40).  It does the same
 * per-byte work as the crate's loop, so it stands in for the crate's COST in
 * the configs[0] baseline and in the default mode's end-to-end record; its
 * boundaries are not the reference's (first cut 5,908 on the KAT input
 * instead of 11,579).
 *
 * Header-only C; used by examples/sf_index.c (-Z) and oracle/sf_baseline.cpp. */
#ifndef ZPAQ_STANDIN_H
#define ZPAQ_STANDIN_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

typedef struct sf_zpaq {
    uint32_t h;
    uint32_t c1;
    uint32_t limit;    /* 2^(32 - bits) */
    uint32_t max_size; /* forced boundary */
    uint64_t run;      /* bytes of the current chunk so far */
    uint8_t o1[256];
} sf_zpaq;

static inline void sf_zpaq_reset(sf_zpaq *z) {
    z->h = 0;
    z->c1 = 0;
    z->run = 0;
    memset(z->o1, 0, sizeof z->o1);
}

static inline void sf_zpaq_init(sf_zpaq *z, unsigned bits, uint32_t max_size) {
    z->limit = bits >= 32 ? 1u : 1u << (32 - bits);
    z->max_size = max_size;
    sf_zpaq_reset(z);
}

/* Bytes of p[0, n) up to and including the next boundary, or 0 if the chunk
 * goes on past p + n.  The state is reset after a boundary. */
static inline size_t sf_zpaq_next(sf_zpaq *z, const uint8_t *p, size_t n) {
    /* state in locals (the crate's &mut self fields do not alias the input;
     * through z every byte store to o1 would reload h, c1 and limit) */
    uint32_t h = z->h, c1 = z->c1;
    const uint32_t limit = z->limit;
    uint8_t o1[256];
    memcpy(o1, z->o1, sizeof o1);
    const uint64_t room = (uint64_t)z->max_size - z->run; /* >= 1 */
    const size_t m = (uint64_t)n < room ? n : (size_t)room;
    for (size_t i = 0; i < m; i++) {
        const uint32_t c = p[i];
        h = (h + c + 1u) * (c == o1[c1] ? 314159265u : 271828182u);
        o1[c1] = (uint8_t)c;
        c1 = c;
        if (h < limit) {
            sf_zpaq_reset(z);
            return i + 1;
        }
    }
    memcpy(z->o1, o1, sizeof o1);
    if ((uint64_t)m == room) { /* the chunk reached max_size */
        sf_zpaq_reset(z);
        return m;
    }
    z->h = h;
    z->c1 = c1;
    z->run += m;
    return 0;
}

#endif /* ZPAQ_STANDIN_H */
