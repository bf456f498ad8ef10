/* zpaq_standin_ops.c -- the stand-in chunker of zpaq_standin.h (timing
 * only: the crate's per-byte work, not its boundaries) as sf_chunker_ops, in
 * a shared library of its own (examples/build/libzpaq_standin.so), so that a
 * caller that cannot include the header -- the Python tests of sf_cut_fd --
 * can hand it to the library.  A Rust caller wraps cdchunking's ZPAQ the same
 * way. */
#include <stdlib.h>

#include "syncfast_amd.h"
#include "zpaq_standin.h"

typedef struct {
    unsigned bits;
    uint32_t max_size;
} standin_cfg;

static void *standin_create(void *ctx) {
    const standin_cfg *c = ctx;
    sf_zpaq *z = malloc(sizeof *z);
    if (z) sf_zpaq_init(z, c->bits, c->max_size);
    return z;
}

static size_t standin_next(void *ch, const uint8_t *p, size_t n) { return sf_zpaq_next(ch, p, n); }

static void standin_destroy(void *ch) { free(ch); }

/* ops for Chunker::new(ZPAQ::new(bits)).max_size(max_size)'s stand-in; the
 * returned table lives until sf_zpaq_standin_ops_free. */
sf_chunker_ops *sf_zpaq_standin_ops(unsigned bits, uint32_t max_size) {
    sf_chunker_ops *ops = malloc(sizeof *ops);
    standin_cfg *cfg = malloc(sizeof *cfg);
    if (!ops || !cfg) {
        free(ops);
        free(cfg);
        return NULL;
    }
    cfg->bits = bits;
    cfg->max_size = max_size ? max_size : 1;
    ops->create = standin_create;
    ops->next = standin_next;
    ops->destroy = standin_destroy;
    ops->ctx = cfg;
    return ops;
}

void sf_zpaq_standin_ops_free(sf_chunker_ops *ops) {
    if (!ops) return;
    free(ops->ctx);
    free(ops);
}
