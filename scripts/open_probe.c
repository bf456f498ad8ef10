/* open_probe.c -- cost of open() + fstat() + close() of many small files,
 * on 1 and on N threads, in a given directory (the default-mode many-file
 * route opens every file once).
 * usage: open_probe DIR NFILES THREADS */
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

static const char *dir;
static int nfiles, nthreads;
static volatile int next_file;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void *worker(void *arg) {
    (void)arg;
    char p[512];
    for (;;) {
        const int k = __sync_fetch_and_add(&next_file, 1);
        if (k >= nfiles) break;
        snprintf(p, sizeof p, "%s/o%06d", dir, k);
        const int fd = open(p, O_RDONLY);
        struct stat sb;
        if (fd >= 0) {
            fstat(fd, &sb);
            close(fd);
        }
    }
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    dir = argv[1];
    nfiles = atoi(argv[2]);
    nthreads = atoi(argv[3]);
    char p[512];
    for (int k = 0; k < nfiles; k++) {
        snprintf(p, sizeof p, "%s/o%06d", dir, k);
        FILE *f = fopen(p, "wb");
        if (!f) return 1;
        fputs("x", f);
        fclose(f);
    }
    for (int pass = 0; pass < 2; pass++) {
        next_file = 0;
        pthread_t th[256];
        const double t0 = now_s();
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, NULL);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
        const double dt = now_s() - t0;
        printf("{\"dir\": \"%s\", \"files\": %d, \"threads\": %d, \"pass\": %d, \"s\": %.4f, \"us_per_open\": %.2f}\n",
               dir, nfiles, nthreads, pass, dt, dt / nfiles * 1e6);
    }
    for (int k = 0; k < nfiles; k++) {
        snprintf(p, sizeof p, "%s/o%06d", dir, k);
        unlink(p);
    }
    return 0;
}
