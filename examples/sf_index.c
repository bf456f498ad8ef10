/* sf_index.c -- a plain-C consumer of the C-ABI (include/syncfast_amd.h).
 *
 * What the Rust side of syncfast would do through its extern "C" binding
 * (INTEGRATION.md), with no Python and no PyTorch: index each path given on
 * the command line with fixed-size blocks and print, per file, its rows as
 * "offset size sha1hex" and its blocks_hash -- the rows Index::index_file
 * inserts (src/index.rs:636-642) and the value compute_blocks_hash stores
 * (src/index.rs:649-682).  Regular files go through sf_index_file, anything
 * else (a FIFO, "-" for stdin) through sf_index_fd.
 *
 *   cc -O2 -I include examples/sf_index.c -L syncfast_amd/lib -lsyncfast_amd \
 *      -Wl,-rpath,$PWD/syncfast_amd/lib -o sf_index
 *   ./sf_index [-b block_size] path...
 */
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "syncfast_amd.h"

static void hex(const uint8_t *d, char out[41]) {
    static const char digits[] = "0123456789abcdef";
    for (int i = 0; i < 20; i++) {
        out[2 * i] = digits[d[i] >> 4];
        out[2 * i + 1] = digits[d[i] & 15];
    }
    out[40] = 0;
}

static int print_rows(const char *name, const sf_block_sig *rows, uint64_t n, const uint8_t bh[20]) {
    char h[41];
    printf("file %s blocks %llu\n", name, (unsigned long long)n);
    for (uint64_t i = 0; i < n; i++) {
        hex(rows[i].sha1, h);
        printf("%llu %u %s\n", (unsigned long long)rows[i].offset, rows[i].size, h);
    }
    hex(bh, h);
    printf("blocks_hash %s\n", h);
    return 0;
}

static int index_one(const char *path, uint32_t bs) {
    uint8_t bh[20];
    struct stat sb;
    const int is_stdin = strcmp(path, "-") == 0;
    if (!is_stdin && stat(path, &sb) == 0 && S_ISREG(sb.st_mode)) {
        uint64_t cap = sb.st_size ? ((uint64_t)sb.st_size + bs - 1) / bs : 0, n = 0;
        sf_block_sig *rows = malloc((cap ? cap : 1) * sizeof(sf_block_sig));
        if (!rows) return SF_ENOMEM;
        int rc = sf_index_file(path, bs, rows, cap, &n, bh);
        if (rc == SF_ENOSPC) {  /* the file grew since stat(): retry with the need */
            sf_block_sig *more = realloc(rows, (n ? n : 1) * sizeof(sf_block_sig));
            if (!more) { free(rows); return SF_ENOMEM; }
            rows = more;
            cap = n;
            rc = sf_index_file(path, bs, rows, cap, &n, bh);
        }
        if (rc == SF_OK) print_rows(path, rows, n, bh);
        free(rows);
        return rc;
    }
    const int fd = is_stdin ? 0 : open(path, O_RDONLY);
    if (fd < 0) return SF_EIO;
    sf_block_sig *rows = NULL;
    uint64_t n = 0;
    const int rc = sf_index_fd(fd, bs, &rows, &n, bh);
    if (!is_stdin) close(fd);
    if (rc == SF_OK) print_rows(path, rows, n, bh);
    sf_free_rows(rows);
    return rc;
}

int main(int argc, char **argv) {
    uint32_t bs = 4096;
    int i = 1;
    if (i + 1 < argc && strcmp(argv[i], "-b") == 0) {
        bs = (uint32_t)strtoul(argv[i + 1], NULL, 10);
        i += 2;
    }
    if (i >= argc) {
        fprintf(stderr, "usage: %s [-b block_size] path...\n", argv[0]);
        return 2;
    }
    int ndev = 0;
    sf_device_count(&ndev);
    if (ndev == 0) {
        fprintf(stderr, "%s: no HIP device (syncfast_amd has no CPU path)\n", argv[0]);
        return 1;
    }
    int status = 0;
    for (; i < argc; i++) {
        const int rc = index_one(argv[i], bs);
        if (rc != SF_OK) {
            fprintf(stderr, "%s: %s\n", argv[i], sf_strerror(rc));
            status = 1;
        }
    }
    sf_release_host_cache();
    return status;
}
