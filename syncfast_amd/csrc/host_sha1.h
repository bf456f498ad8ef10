// host_sha1.h -- library-internal host SHA-1 entry points (host_sha1.cpp).
// Not part of the C-ABI in include/syncfast_amd.h.
#pragma once
#include <stdint.h>

extern "C" {
void sf_host_sha1_impl(const uint8_t* data, uint64_t len, uint8_t out[20], int force_scalar);
int sf_host_has_shani(void);

struct sf_host_sha1_stream {
  uint32_t h[5];
  uint8_t buf[64];
  uint32_t nbuf;
  uint64_t total;
  int shani;
};
void sf_host_sha1_begin(sf_host_sha1_stream* s);
void sf_host_sha1_update(sf_host_sha1_stream* s, const uint8_t* p, uint64_t n);
void sf_host_sha1_final(sf_host_sha1_stream* s, uint8_t out[20]);
}
