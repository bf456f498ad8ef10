// sf_kernels.hpp -- the MI355X block-signature kernels (device code, included by sf_capi.hip).
//
// Replaces the hot loop of Index::index_file, /root/reference/src/index.rs:
// 629-647 (SHA-1 of every block; `Sha1::update` / `digest` / `reset`) and is
// reused for compute_blocks_hash (src/index.rs:661-682) of many files at once.
//
// Design (DESIGN.md "Kernels"):
//   * one LANE per block: SHA-1 is sequential inside a message, so a block is
//     a lane's private message and a wave hashes 64 blocks in lockstep;
//   * a wave's 64 blocks are streamed through a per-wave LDS tile of
//     64 blocks x TILE bytes, filled by LDS-DMA (`buffer_load_dwordx4 ... lds`):
//     every DMA wave-instruction moves TILE/16 full 16-B pieces of 1024/TILE
//     blocks, so each instruction reads whole 128-B lines; the piece order is
//     XOR-swizzled on the SOURCE address so that the per-lane `ds_read_b128`
//     of a block's own pieces is bank-conflict free;
//   * the tile for step t+1 is issued right after step t's words are in
//     registers, so one DMA per wave is always in flight behind TILE/64
//     compressions of VALU work;
//   * the final (padding) chunk(s) of each block are built with per-lane,
//     bounds-checked loads, so nothing is ever read outside [0, len).
// Buffer resources carry num_records = bytes left in the wave's span, so a
// DMA lane past the end reads zeros instead of faulting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/syncfast_amd.h"
#include "sf_chain.hpp"

namespace sf {

constexpr int kWave = 64;
constexpr int kWavesPerWG = 4;
constexpr int kThreads = kWave * kWavesPerWG;
constexpr uint32_t kRsrcWord3 = 0x00020000u;  // raw buffer, gfx9 family

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// ---------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// A value identical in every lane, moved to SGPRs so that everything derived
// from it (buffer resources, loop bounds) stays scalar.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, m, 64));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m, 64));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = __shfl_xor((unsigned long long)v, m, 64);
    v = o < v ? o : v;
  }
  return uniform_u64(v);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = __shfl_xor((unsigned long long)v, m, 64);
    v = o > v ? o : v;
  }
  return uniform_u64(v);
}

// 64 bytes at any byte address (four 16-B loads; unaligned global access).
__device__ __forceinline__ void ld_chunk_any(uint4 (&v)[4], const uint8_t* p) {
#pragma unroll
  for (int q = 0; q < 4; ++q) __builtin_memcpy(&v[q], p + 16 * q, 16);
}

// 64 bytes at a 4-B aligned address (four 16-B loads).
__device__ __forceinline__ void ld_chunk_al(uint4 (&v)[4], const uint32_t* p) {
#pragma unroll
  for (int k = 0; k < 4; ++k) __builtin_memcpy(&v[k], p + 4 * k, 16);
}

// K_t + W_t of the padding-only chunk ending a block of `bytes` bytes
// (bytes % 64 == 0), filled by the host (sf_capi.hip) and passed by value.
struct PadSchedule {
  uint32_t bytes;  // 0 = not available
  uint32_t kw[80];
};

// Per-wave geometry of the blocks handled by this wave.
struct WaveGeo {
  uint64_t base;      // byte offset of the wave's span in `data`
  uint64_t span;      // bytes in [base, end of last block)
  uint32_t min_size;  // min block size over valid lanes
  uint32_t max_size;  // max block size over valid lanes
  uint32_t max_nch;   // max compressions over valid lanes
  bool lds_ok;        // 16-B aligned pieces and span < 4 GiB
};

// Cache policy of the aligned path's LDS-DMA: nt, the input is streamed once
// (+1.4 % in A/B, profiles/r01/tune_sched_nt.log).
constexpr int kLoadAux = 2;

// Issue the LDS-DMA fill of step `step` (bytes [step*TILE, step*TILE+TILE) of
// every block) into the wave's tile.  The buffer resource starts at the step
// and covers the rest of the span, so lanes past the span read zeros.
template <int TILE>
__device__ __forceinline__ void issue_step(const uint8_t* span_ptr, uint64_t span, uint32_t step,
                                           const uint32_t* voff, uint4* wave_tile) {
  // All operands are wave-uniform; readfirstlane keeps the resource in SGPRs
  // (a VGPR resource makes hipcc wrap every DMA in a waterfall loop).
  const uint64_t toff = (uint64_t)step * TILE;
  const uint64_t left = span > toff ? span - toff : 0;
  const uint32_t nrec = __builtin_amdgcn_readfirstlane(left > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)left);
  const uint64_t ptr = uniform_u64(reinterpret_cast<uint64_t>(span_ptr + toff));
  __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ptr), (short)0, (int)nrec, (int)kRsrcWord3);
#pragma unroll
  for (int j = 0; j < TILE / 16; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(wave_tile + j * 64), 16, voff[j], 0, 0, kLoadAux);
}

// Hash the block (off, size) owned by this lane; all 64 lanes of the wave
// enter together.  `rel` = off - geo.base (valid lanes).  TILE = bytes of
// each block staged per LDS step.  WEAK: also fold the same words into the
// lane's Adler-32 (opt-in weak sum, sha1_device.hpp).
template <int TILE, bool HAS_PAD, bool WEAK = false>
__device__ __forceinline__ void hash_wave(const uint8_t* __restrict__ data, uint64_t off, uint32_t size,
                                          uint32_t rel, bool valid, const WaveGeo& geo,
                                          uint4* __restrict__ wave_tile, Sha1& st, const PadSchedule pad,
                                          Adler& wk) {
  constexpr int PIECES = TILE / 16;           // 16-B pieces per block per step
  constexpr int CH = TILE / 64;               // compressions per step
  constexpr int GSHIFT = PIECES == 4 ? 2 : (PIECES == 8 ? 1 : 0);
  constexpr int BLK_PER_DMA = 1024 / TILE;    // blocks covered by one DMA wave-instruction
  static_assert(PIECES == 4 || PIECES == 8 || PIECES == 16, "TILE must be 64, 128 or 256");
  const int lane = lane_id();

  st.init();
  if constexpr (WEAK) wk.init();
  const uint32_t nfull = geo.min_size / 64u;
  uint32_t c_done = 0;  // this lane's chunks done
  if (geo.lds_ok) {
    const uint32_t nsteps = nfull / CH;
    // Source offsets (relative to the span base) of this lane's 16-B piece in
    // each of the PIECES DMA instructions of one step.  Instruction j writes
    // LDS bytes [j*1024, j*1024+1024): lane -> block b, slot s; slot s holds
    // piece k = s ^ g(b) so that the reads below are conflict free.
    uint32_t voff[PIECES];
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      const int b = j * BLK_PER_DMA + lane / PIECES;
      const int s = lane % PIECES;
      const int k = s ^ ((b >> GSHIFT) & (PIECES - 1));
      const uint32_t rel_b = (uint32_t)__shfl((int)rel, b, 64);
      voff[j] = rel_b + (uint32_t)k * 16u;
    }
    const int g = (lane >> GSHIFT) & (PIECES - 1);
    const uint4* my = wave_tile + lane * PIECES;
    const uint8_t* span_ptr = data + geo.base;

    if (nsteps > 0) issue_step<TILE>(span_ptr, geo.span, 0, voff, wave_tile);
    for (uint32_t t = 0; t < nsteps; ++t) {
      uint4 raw[PIECES];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < PIECES; ++k) raw[k] = my[k ^ g];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 1 < nsteps) issue_step<TILE>(span_ptr, geo.span, t + 1, voff, wave_tile);
#pragma unroll
      for (int ch = 0; ch < CH; ++ch) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v = raw[ch * 4 + q];
          w[4 * q + 0] = bswap32(v.x);
          w[4 * q + 1] = bswap32(v.y);
          w[4 * q + 2] = bswap32(v.z);
          w[4 * q + 3] = bswap32(v.w);
        }
        if constexpr (WEAK) {
          uint32_t le[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint4 v = raw[ch * 4 + q];
            le[4 * q + 0] = v.x;
            le[4 * q + 1] = v.y;
            le[4 * q + 2] = v.z;
            le[4 * q + 3] = v.w;
          }
          wk.chunk(le);
        }
        st.compress(w);
      }
    }
    c_done = nsteps * CH;
  } else {
    if constexpr (HAS_PAD) {
      // (fixed tiling, only for a misaligned data pointer or block size: the
      // hot kernel's code -- any change here moves its register assignment,
      // and one such move cost the headline launch 3.7 %)
      // Misaligned or > 4 GiB span: each lane streams its own block, 64 B per
      // compression with four (unaligned) 16-B loads, the next chunk's loads
      // in flight while the current one is compressed.
      const uint8_t* p = data + off;
      uint4 nx[4];
      if (nfull) ld_chunk_any(nx, p);
      for (uint32_t c = 0; c < nfull; ++c) {
        uint32_t le[16], w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          le[4 * q + 0] = nx[q].x;
          le[4 * q + 1] = nx[q].y;
          le[4 * q + 2] = nx[q].z;
          le[4 * q + 3] = nx[q].w;
        }
        if (c + 1 < nfull) ld_chunk_any(nx, p + (uint64_t)(c + 1) * 64);
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap32(le[j]);
        if constexpr (WEAK) wk.chunk(le);
        st.compress(w);
      }
      c_done = nfull;
    } else {
      // Misaligned or > 4 GiB span: each lane streams its own block, 64 B per
      // compression, the next chunk's loads in flight while the current one is
      // compressed, up to ITS OWN last whole chunk (lanes whose block has fewer
      // whole chunks than the wave's longest idle meanwhile).  Loads are
      // dword-aligned (a byte-aligned 16-B load costs the address unit several
      // times over: 4 KiB blocks at byte offset +1 ran at 1911 GiB/s, at +4 at
      // 2832, scripts/ragged_probe.py): the lane reads 17 dwords from its block
      // start rounded down to 4 B and shifts the message words out of them
      // (v_alignbyte by the lane's byte offset r).  Every dword read holds at
      // least one byte of the block, so nothing is touched outside the dwords
      // the block's bytes lie in.
      const uint8_t* p = data + off;
      const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
      const uint32_t* q = reinterpret_cast<const uint32_t*>(p - r);
      const uint32_t mine = valid ? size / 64u : 0u;  // this lane's whole chunks
      const uint32_t upto = geo.max_size / 64u;       // the wave's most
      uint4 nx[4];
      uint32_t nx16 = 0u;  // dword 16 of the chunk in nx (needed when r != 0)
      if (mine) {
        ld_chunk_al(nx, q);
        if (r != 0u || mine > 1) nx16 = q[16];
      }
      for (uint32_t c = 0; c < upto; ++c) {
        if (c < mine) {
          uint32_t d[17], le[16], w[16];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            d[4 * k + 0] = nx[k].x;
            d[4 * k + 1] = nx[k].y;
            d[4 * k + 2] = nx[k].z;
            d[4 * k + 3] = nx[k].w;
          }
          d[16] = nx16;
          if (c + 1 < mine) {
            ld_chunk_al(nx, q + 16 * (uint64_t)(c + 1));
            if (r != 0u || c + 2 < mine) nx16 = q[16 * (uint64_t)(c + 2)];
          }
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            le[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], r);
            w[j] = bswap32(le[j]);
          }
          if constexpr (WEAK) wk.chunk(le);
          st.compress(w);
        }
      }
      c_done = mine;
    }
  }
  // Weak sum of this lane's bytes past the chunks both paths consumed
  // (whole chunks, then < 64 single bytes); never reads outside the block.
  if constexpr (WEAK) {
    if (valid) {
      const uint8_t* p = data + off;
      const uint32_t full = size / 64u;
      for (uint32_t c = c_done; c < full; ++c) {
        uint32_t le[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) le[j] = ld_u32_any(p + (uint64_t)c * 64 + 4 * j);
        wk.chunk(le);
      }
      for (uint32_t i = full * 64u; i < size; ++i) wk.byte(p[i]);
    }
  }
  // Every block of the wave has the same 64-B multiple size and all its data
  // chunks are done: the last chunk is the same padding for every lane.
  // (pad is passed by value, never by address: a kernel argument whose
  // address escapes is copied to scratch.)
  if (HAS_PAD && pad.bytes == geo.min_size && geo.min_size == geo.max_size && c_done == nfull) {
    st.compress_uniform(pad.kw);
    return;
  }
  // Remaining data chunks and the padding chunk(s), per lane.
  if constexpr (HAS_PAD) {
    const uint32_t nch = n_chunks(size);
    for (uint32_t c = c_done; c < geo.max_nch; ++c) {
      if (valid && c < nch) {
        uint32_t w[16];
        build_tail_chunk(w, data + off, size, c, nch);
        st.compress(w);
      }
    }
  } else {
    // An explicit list's block may be any uint32 size: the index of its last
    // chunk, (size + 8) / 64, without the 32-bit wrap of n_chunks from
    // 2^32 - 8.
    const uint32_t last = (size >> 6) + ((size & 63u) >= 56u ? 1u : 0u);
    for (uint32_t c = c_done; c < geo.max_nch; ++c) {
      if (valid && c <= last) {
        uint32_t w[16];
        build_tail_chunk(w, data + off, size, c, last + 1u);
        st.compress(w);
      }
    }
  }
}

// ---------------------------------------------------------------- kernels

// Fixed tiling: block i = data[i*bs, min((i+1)*bs, len)).  One workgroup
// `group` of it (4 waves x 64 consecutive blocks): the body of
// sha1_fixed_kernel and of the block part of sha1_fixed_chained_kernel.
template <int TILE, bool WEAK>
__device__ __forceinline__ void fixed_wave(const uint8_t* __restrict__ data, uint64_t len, uint32_t bs,
                                           uint64_t nblocks, uint8_t* __restrict__ digests, const PadSchedule pad,
                                           uint32_t* __restrict__ weak, uint64_t wave, uint4* __restrict__ tile) {
  const int lane = lane_id();
  const uint64_t first = wave * 64;  // this wave's 64 consecutive blocks
  if (first >= nblocks) return;
  const uint64_t blk = first + lane;
  const bool valid = blk < nblocks;
  const uint64_t off = valid ? blk * bs : first * bs;
  const uint32_t size = valid ? (uint32_t)(len - off < bs ? len - off : bs) : 0u;

  WaveGeo geo;
  geo.base = first * bs;
  const uint64_t last = (first + 64 <= nblocks) ? first + 63 : nblocks - 1;
  geo.span = len - geo.base < (last - first + 1) * (uint64_t)bs ? len - geo.base : (last - first + 1) * (uint64_t)bs;
  const uint32_t last_size = (uint32_t)(len - last * bs < bs ? len - last * bs : bs);
  geo.min_size = last_size < bs ? last_size : bs;
  geo.max_size = bs;
  geo.max_nch = n_chunks(bs);
  geo.lds_ok = ((bs & 15u) == 0) && ((reinterpret_cast<uintptr_t>(data) & 15u) == 0) &&
               (64ull * bs < 0xF0000000ull);
  const uint32_t rel = (uint32_t)((uint64_t)lane * bs);

  Sha1 st;
  Adler wk;
  hash_wave<TILE, true, WEAK>(data, off, size, rel, valid, geo, tile, st, pad, wk);
  if (valid) {
    st.store(digests + blk * 20);
    if constexpr (WEAK) weak[blk] = wk.fin();
  }
}

// WPE = minimum resident waves per SIMD requested from the register
// allocator (__launch_bounds__ 2nd argument, per EU on gfx950).
template <int TILE, int WPE = 1, bool WEAK = false>
__global__ void __launch_bounds__(kThreads, WPE)
sha1_fixed_kernel(const uint8_t* __restrict__ data, uint64_t len, uint32_t bs, uint64_t nblocks,
                  uint8_t* __restrict__ digests, const PadSchedule pad, uint32_t* __restrict__ weak) {
  __shared__ uint4 smem[kWavesPerWG * 64 * (TILE / 16)];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform -> SGPR
  fixed_wave<TILE, WEAK>(data, len, bs, nblocks, digests, pad, weak, (uint64_t)blockIdx.x * kWavesPerWG + wid,
                         smem + wid * 64 * (TILE / 16));
}

// Stream a 64-B-multiple byte range [lo, hi) of a lane's message through
// SHA-1, the next chunk's loads issued before each compression (the load
// has a whole compression to land; one register set keeps the VGPR count
// under the block kernel's when fused with it).
__device__ __forceinline__ void sha1_stream_range(Sha1& st, const uint4* __restrict__ q, uint32_t lo, uint32_t hi) {
  if (lo + 64 > hi) return;
  uint4 c0 = q[lo / 16], c1 = q[lo / 16 + 1], c2 = q[lo / 16 + 2], c3 = q[lo / 16 + 3];
  for (uint32_t c = lo; c + 64 <= hi; c += 64) {
    const uint32_t nx = (c + 128 <= hi) ? (c + 64) / 16 : c / 16;
    const uint4 n0 = q[nx], n1 = q[nx + 1], n2 = q[nx + 2], n3 = q[nx + 3];
    __builtin_amdgcn_sched_barrier(0);
    uint32_t w[16] = {bswap32(c0.x), bswap32(c0.y), bswap32(c0.z), bswap32(c0.w),
                      bswap32(c1.x), bswap32(c1.y), bswap32(c1.z), bswap32(c1.w),
                      bswap32(c2.x), bswap32(c2.y), bswap32(c2.z), bswap32(c2.w),
                      bswap32(c3.x), bswap32(c3.y), bswap32(c3.z), bswap32(c3.w)};
    st.compress(w);
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
}

// One lane per file: the file's blocks_hash (src/index.rs:661-682) = SHA-1
// over its run of run_len digest bytes (the stand-alone chain kernel).
__device__ __forceinline__ void chain_wave(const uint8_t* __restrict__ runs, uint64_t run_stride, uint32_t f,
                                           bool valid, uint32_t run_len, uint8_t* __restrict__ out) {
  if (!valid) return;
  Sha1 st;
  st.init();
  const uint8_t* p = runs + (uint64_t)f * run_stride;
  sha1_stream_range(st, reinterpret_cast<const uint4*>(p), 0, (run_len / 64) * 64);
  const uint32_t nch = n_chunks(run_len);
  for (uint32_t c = run_len / 64; c < nch; ++c) {
    uint32_t w[16];
    build_tail_chunk(w, p, run_len, c, nch);
    st.compress(w);
  }
  st.store(out + (uint64_t)f * 20);
}

#ifndef SF_STREAM_TU  // kernels of sf_capi.hip only (sf_stream.hip includes the device functions)
// Stand-alone chains (no stages): one lane per file over its whole run.
__global__ void __launch_bounds__(64)
sha1_chain_kernel(const uint8_t* __restrict__ runs, uint64_t run_stride, uint32_t nfiles, uint32_t run_len,
                  uint8_t* __restrict__ out) {
  const uint32_t f = blockIdx.x * 64 + threadIdx.x;
  chain_wave(runs, run_stride, f, f < nfiles, run_len, out);
}
#endif

constexpr int kChainPrio = 3;  // wave priority of the stream's chain waves
// A stream's chain job on the chain wave of a block launch (wave 0 of one
// of the first workgroups, sha1_fixed_chained_kernel).  Its digest loads are
// staged through the workgroup's LDS tile (unused by a chain wave
// otherwise), as the block waves stage theirs: per step, 8 DMA
// wave-instructions each move whole 128-B lines of 8 files, so one
// instruction touches 8 lines instead of the 64 that a lane-per-file load
// touches.  The lane-per-file loads (4 chunks in flight per lane) cost the
// launch 0.050 ms per batch of chains, the staged form 0.032 (config 3
// launch sequence, profiles/r03/c3/seq/seq_chain_lds.txt).  Data chunks
// [lo, hi) of each lane's run; part 0/2 then the padding chunk(s).
__device__ __forceinline__ void chain_job(const ChainJob& j, uint32_t wave, uint4* __restrict__ tile) {
  __builtin_amdgcn_s_setprio(kChainPrio);  // latency-bound chains issue first on a shared SIMD
  const int lane = lane_id();
  const uint32_t f = wave * 64 + lane;
  const bool valid = f < j.files;
  Sha1 st;
  if (j.part == 2 && valid) {
    const uint32_t* sv = reinterpret_cast<const uint32_t*>(j.state + (uint64_t)f * 20);
    st.h0 = sv[0]; st.h1 = sv[1]; st.h2 = sv[2]; st.h3 = sv[3]; st.h4 = sv[4];
  } else {
    st.init();
  }
  const uint32_t n = j.hi - j.lo;                 // data chunks, uniform
  const uint32_t nsteps = (n + 1) / 2;
  const uint8_t* span_ptr = j.runs + (uint64_t)wave * 64 * j.run_len + (uint64_t)j.lo * 64;
  const uint64_t files_here = j.files - wave * 64 < 64 ? j.files - wave * 64 : 64;
  const uint64_t span = (files_here - 1) * j.run_len + (uint64_t)n * 64;
  uint32_t voff[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int b = q * 8 + lane / 8;  // file of the wave
    const int s = lane % 8;
    const int k = s ^ ((b >> 1) & 7);
    voff[q] = (uint32_t)b * j.run_len + (uint32_t)k * 16u;
  }
  const int g = (lane >> 1) & 7;
  const uint4* my = tile + lane * 8;
  if (nsteps > 0) issue_step<128>(span_ptr, span, 0, voff, tile);
  for (uint32_t t = 0; t < nsteps; ++t) {
    uint4 raw[8];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) raw[k] = my[k ^ g];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 1 < nsteps) issue_step<128>(span_ptr, span, t + 1, voff, tile);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      if (2 * t + ch < n) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          w[4 * i + 0] = bswap32(raw[4 * ch + i].x);
          w[4 * i + 1] = bswap32(raw[4 * ch + i].y);
          w[4 * i + 2] = bswap32(raw[4 * ch + i].z);
          w[4 * i + 3] = bswap32(raw[4 * ch + i].w);
        }
        st.compress(w);
      }
    }
  }
  if (!valid) return;
  const uint8_t* p = j.runs + (uint64_t)f * j.run_len;
  if (j.part == 1) {
    uint32_t* sv = reinterpret_cast<uint32_t*>(j.state + (uint64_t)f * 20);
    sv[0] = st.h0; sv[1] = st.h1; sv[2] = st.h2; sv[3] = st.h3; sv[4] = st.h4;
    return;
  }
  const uint32_t nch = n_chunks(j.run_len);
  for (uint32_t c = j.run_len / 64; c < nch; ++c) {
    uint32_t w[16];
    build_tail_chunk(w, p, j.run_len, c, nch);
    st.compress(w);
  }
  st.store(j.hashes + (uint64_t)f * 20);
}

// sha1_fixed_chained_kernel (a stream's batches with their chains) is in
// sf_stream.hip, its own translation unit.

// ------------------------------------------- explicit lists at any offset
// The reference's default blocks are content-defined (cdchunking ZPAQ,
// src/index.rs:622-625): they start at any byte.  A wave of such blocks still
// stages them through LDS by DMA (round 3):
//   * step t stages 9 pieces of 16 B of every block, [a + 128t, a + 128t +
//     144) with a = off rounded down to 4 B (the DMA takes any dword-aligned
//     source), which holds the block's message bytes [off + 128t, off + 128t
//     + 128) whatever off & 3 is;
//   * a block's 9 pieces sit back to back in LDS (144-B slots, 9 KiB per
//     wave), so one DMA wave-instruction reads ~7 blocks x 144 contiguous
//     bytes, and with a slot stride of 9 quads the lanes' ds_read_b128 are
//     conflict-free;
//   * one v_perm per word shifts by off & 3 and byte-swaps at once (selector
//     in a VGPR): as many VALU as the aligned path's plain byte swap;
//   * a lane's last chunks (the partial one with the 0x80 byte, and the
//     length) are built from the same LDS words, so no lane issues a global
//     load of its own; chunks past a lane's message are skipped (exec mask),
//     which in a length-sorted wave costs ~1 chunk of 130.
// Each 128-B line of a block is touched by two consecutive steps (the window
// is 144 B and advances 128 B); the second touch is an L2 hit ~80 % of the
// time with the default cache policy (PMC: 1.21x the algorithmic bytes).
// With nt on every piece it was 1.95x; nt on the first 8 pieces and the
// default on the 9th (a 9th DMA instruction) 1.42x, since the 8-piece window
// itself ends in the next line (profiles/r03/).
constexpr int kListPieces = 9;

// Cache policy of the slot DMA: the default (0), not the aligned path's nt
// (see above).
constexpr int kListLoadAux = 0;
template <int NP>
__device__ __forceinline__ void issue_pieces(const uint8_t* span_ptr, uint64_t span4, uint32_t step,
                                             const uint32_t (&voff)[NP], uint4* wave_tile) {
  const uint64_t toff = (uint64_t)step * 128u;
  const uint64_t left = span4 > toff ? span4 - toff : 0;
  const uint32_t nrec = __builtin_amdgcn_readfirstlane(left > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)left);
  const uint64_t ptr = uniform_u64(reinterpret_cast<uint64_t>(span_ptr + toff));
  __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ptr), (short)0, (int)nrec, (int)kRsrcWord3);
#pragma unroll
  for (int j = 0; j < NP; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(wave_tile + j * 64), 16, voff[j], 0, 0,
                                             kListLoadAux);
}

// Words of chunk c of a message of `size` bytes whose data words (already
// big-endian) are in w: keep the rem = size - 64c data bytes, then the 0x80
// byte, zeros, and the bit length if c is the last chunk (nch - 1).
__device__ __forceinline__ void finish_chunk(uint32_t (&w)[16], uint32_t size, uint32_t c, uint32_t nch) {
  // size < 0xF0000000 on the slot path, so c * 64 does not wrap; the
  // difference is taken in uint32 and then read as signed: a padding-only
  // chunk (c * 64 > size) gives a small negative rem for sizes >= 2^31 too
  const int rem = (int)(size - c * 64u);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = rem - 4 * j;  // data bytes in word j
    uint32_t x;
    if (v >= 4) x = w[j];
    else if (v > 0) x = (w[j] & (0xFFFFFFFFu << (32 - 8 * v))) | (0x80u << (24 - 8 * v));
    else if (v == 0) x = 0x80000000u;
    else x = 0u;
    w[j] = x;
  }
  if (c + 1 == nch) {
    w[14] = size >> 29;
    w[15] = size << 3;
  }
}

// A lane's 36 dwords of one step out of its 144-B LDS slot (9 b128 reads;
// a slot stride of 9 quads puts any 16 lanes' reads on 16 distinct bank
// quads).  Per-lane dword reads at (off & 15) >> 2 from 16-B aligned pieces
// were tried first: 4-way bank conflicts, no faster (profiles/r03/).
__device__ __forceinline__ void list_read(uint32_t (&d)[36], const uint4* myq) {
#pragma unroll
  for (int k = 0; k < kListPieces; ++k) {
    const uint4 v = myq[k];
    d[4 * k + 0] = v.x;
    d[4 * k + 1] = v.y;
    d[4 * k + 2] = v.z;
    d[4 * k + 3] = v.w;
  }
}

// Hash this lane's block (off, size) of an explicit list through 144-B LDS
// slots; all 64 lanes enter together.  base = the wave's lowest block start
// rounded down to 16 B; span = bytes from base to the wave's highest block
// end (< 4 GiB); data 16-B aligned.  The DMA is range-checked per dword
// against span rounded up to 4 B: it reads only dwords that hold a byte of
// the wave's span (past it, zeros).
__device__ __forceinline__ void hash_wave_list(const uint8_t* __restrict__ data, uint64_t off, uint32_t size,
                                               bool valid, uint64_t base, uint64_t span, uint4* __restrict__ wave_tile,
                                               Sha1& st) {
  const int lane = lane_id();
  st.init();
  // compressions of this lane's message (the slot path's blocks are < 3.75
  // GiB, so the 32-bit form cannot wrap; the wide form cost 5 spilled VGPRs)
  const uint32_t nch = n_chunks(size);
  const uint32_t mine = valid ? size / 64u : 0u;       // its whole data chunks
  const uint32_t nsteps = wave_max_u32(valid ? (nch + 1u) / 2u : 0u);
  const uint32_t rel = valid ? (uint32_t)((off & ~3ull) - base) : 0u;  // pieces start at the block's dword
  uint32_t voff[kListPieces];
#pragma unroll
  for (int j = 0; j < kListPieces; ++j) {
    const int p = 64 * j + lane;  // piece p of the tile: block p / 9, piece p % 9
    const uint32_t rel_b = (uint32_t)__shfl((int)rel, p / kListPieces, 64);
    voff[j] = rel_b + 16u * (uint32_t)(p % kListPieces);
  }
  const uint4* myq = wave_tile + lane * kListPieces;  // 144-B slots
  const uint32_t sel = 0x00010203u + ((uint32_t)off & 3u) * 0x01010101u;  // shift by off & 3, then byte swap
  const uint8_t* span_ptr = data + base;
  const uint64_t span4 = (span + 3u) & ~3ull;  // range-checked per dword: a dword holding a block byte is read
  // Steps in which every lane has two whole data chunks run branch-free (one
  // basic block per step: the scheduler interleaves the two compressions, as
  // in the aligned path); only the wave's last steps test each lane.
  const uint32_t nfast = wave_min_u32(valid ? mine / 2u : 0xFFFFFFFFu);
  if (nsteps > 0) issue_pieces(span_ptr, span4, 0, voff, wave_tile);
  uint32_t t = 0;
  for (; t < nfast; ++t) {
    uint32_t d[36];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    list_read(d, myq);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 1 < nsteps) issue_pieces(span_ptr, span4, t + 1, voff, wave_tile);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(d[16 * ch + j + 1], d[16 * ch + j], sel);
      st.compress(w);
    }
  }
  for (; t < nsteps; ++t) {
    uint32_t d[36];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    list_read(d, myq);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 1 < nsteps) issue_pieces(span_ptr, span4, t + 1, voff, wave_tile);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      const uint32_t c = 2 * t + ch;
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(d[16 * ch + j + 1], d[16 * ch + j], sel);
      if (c < nch) {
        if (c >= mine) finish_chunk(w, size, c, nch);
        st.compress(w);
      }
    }
  }
}

constexpr int kTableWavesPerSimd = 3;  // waves/SIMD the explicit-list kernel's register budget is sized for
constexpr int kTableWG = 4;             // its waves per workgroup
constexpr uint32_t kTableRound = 1024u; // waves per dispatch round: MI355X's SIMDs (256 CUs x 4)
constexpr uint32_t kTableReversedRounds = 2u;  // bit r: round r takes its groups in reverse (round 1 only)

// Explicit block list: block i = data[offsets[i], offsets[i] + sizes[i]).
// Used for content-defined boundaries, the reference KAT boundaries, ragged
// many-file batches, and (over the digest table) per-file blocks_hash.
// A block outside [0, len) is not read: its digest is zeroed and *status is
// set to -34 (SF_ERANGE).
// Group g of the list = 64 blocks, one lane each: order[64g .. 64g + 63] when
// the launcher sorted the list (each digest is written at the block's own
// index), else blocks 64g .. 64g + 63.
template <int TILE, bool WEAK>
__device__ __forceinline__ void table_group(const uint8_t* __restrict__ data, uint64_t len,
                                            const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ sizes,
                                            uint64_t nblocks, uint8_t* __restrict__ digests, int* __restrict__ status,
                                            uint32_t* __restrict__ weak, const uint32_t* __restrict__ order,
                                            uint64_t g, uint4* __restrict__ tile) {
  const int lane = lane_id();
  const uint64_t first = g * 64;
  bool valid = first + lane < nblocks;
  const uint64_t blk = (order && valid) ? (uint64_t)order[first + lane] : first + lane;
  uint64_t off = 0;
  uint32_t size = 0;
  bool bad = false;
  if (valid) {
    off = offsets[blk];
    size = sizes[blk];
    if (off > len || (uint64_t)size > len - off) {
      bad = true;
      off = 0;
      size = 0;
    }
  }
  WaveGeo geo;
  const uint64_t lo = wave_min_u64(valid ? off : ~0ull);
  const uint64_t hi = wave_max_u64(valid ? off + size : 0ull);
  geo.base = lo;
  geo.span = hi - lo;
  geo.min_size = wave_min_u32(valid ? size : 0xFFFFFFFFu);
  geo.max_size = wave_max_u32(valid ? size : 0u);
  geo.max_nch = wave_max_u32(valid ? n_chunks_wide(size) : 0u);
  const bool aligned = !valid || ((off & 15u) == 0);
  geo.lds_ok = __builtin_amdgcn_readfirstlane(__all(aligned)) &&
               ((reinterpret_cast<uintptr_t>(data) & 15u) == 0) && geo.span < 0xF0000000ull;
  const uint32_t rel = valid ? (uint32_t)(off - lo) : 0u;

  Sha1 st;
  Adler wk;
  // The slot path also takes aligned waves whose blocks differ in size: the
  // aligned path stages only the wave's shortest block's chunks through LDS
  // and loads the rest per lane (a CDC-like list laid out 16-B aligned: 2772
  // GiB/s that way, 3045 through the slots; equal 8 KiB blocks: 3165 aligned,
  // 3138 at byte offsets through the slots; profiles/r03/cdcx/).
  const uint64_t lo16 = lo & ~15ull;
  const bool list_path = !WEAK && (!geo.lds_ok || geo.min_size != geo.max_size) &&
                         ((reinterpret_cast<uintptr_t>(data) & 15u) == 0) && hi - lo16 < 0xF0000000ull;
  if (list_path)
    hash_wave_list(data, off, size, valid, lo16, hi - lo16, tile, st);
  else
    hash_wave<TILE, false, WEAK>(data, off, size, rel, valid, geo, tile, st, PadSchedule{}, wk);
  if (valid) {
    if (bad) {
      uint32_t* o = reinterpret_cast<uint32_t*>(digests + blk * 20);
      o[0] = o[1] = o[2] = o[3] = o[4] = 0;
      if constexpr (WEAK) weak[blk] = 0u;
      if (status) *status = SF_ERANGE;
    } else {
      st.store(digests + blk * 20);
      if constexpr (WEAK) weak[blk] = wk.fin();
    }
  }
}

// The explicit-list kernel: wave w of the grid hashes group w (one group of
// 64 blocks per wave, kTableWG waves per workgroup).  How the waves of a
// sorted list are scheduled decides its rate (DESIGN.md section 3.4, round
// 4, where the per-wave traces and the persistent forms measured against it
// are recorded):
//   * the sequencer issues the OLDEST wave of a SIMD first, so a wave that
//     starts first -- with the sort, one of the longest groups -- runs at
//     nearly the rate it would alone (1.33 us per compression beside two
//     other waves, the 4 KiB list's waves 2.9 us), and the younger waves
//     fill its gaps: hardware dispatch in the sort's order already gives the
//     longest groups the critical path;
//   * persistent waves that claim groups from a counter lose that: a wave's
//     age is its launch, not its group's, so an old wave that keeps claiming
//     groups starves a younger neighbour, whose group then ends last;
//   * what is left is the end of the launch, and most of it is set by the
//     first round: waves w, w + 1024 and w + 2048 land on one SIMD, so in
//     the sort's order the same SIMDs would start with every round's
//     longest group.  Round 1 therefore takes its groups in reverse (below):
//     SIMD work max/mean 1.07 -> 1.047, the CDC-like list 2 % faster.
template <int TILE, bool WEAK = false>
__global__ void __launch_bounds__(64 * kTableWG, kTableWavesPerSimd)
sha1_table_kernel(const uint8_t* __restrict__ data, uint64_t len, const uint64_t* __restrict__ offsets,
                  const uint32_t* __restrict__ sizes, uint64_t nblocks, uint8_t* __restrict__ digests,
                  int* __restrict__ status, uint32_t* __restrict__ weak, const uint32_t* __restrict__ order) {
  constexpr int kWaveTile = 64 * (TILE / 16) > 64 * kListPieces ? 64 * (TILE / 16) : 64 * kListPieces;
  __shared__ uint4 smem[kTableWG * kWaveTile];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint4* tile = smem + wid * kWaveTile;
  const uint32_t ngroups = (uint32_t)((nblocks + 63) / 64);  // <= 2^25: the launcher splits at 2^31 blocks
  uint32_t g = blockIdx.x * kTableWG + wid;
  // The first rounds of waves land one per SIMD per round (wave w and
  // w + kTableRound on the same SIMD, traces of round 4), so in the sort's
  // order SIMD i would start with groups i, R + i and 2R + i: the longest
  // group of every round on the same SIMDs (first-round work per SIMD
  // 589..967 compressions, mean 764, on the CDC-like list).  Round 1 takes
  // its groups in reverse, pairing the longest of round 0 with the shortest
  // of round 1.  R is MI355X's 1024 SIMDs at compile time: a runtime R moved
  // this kernel's compiled form and cost the 4 KiB list 6 % (profiles/r04/s18/);
  // on a device with fewer SIMDs (a CPX/QPX partition) the reversal is one
  // harmless permutation of round 1 whose gain does not carry over.
  if (order) {
    const uint32_t R = kTableRound, r = g / R;
    if (r < 8 && ((kTableReversedRounds >> r) & 1u) && (r + 1) * R <= ngroups) g = r * R + (R - 1u - g % R);
  }
  if (g < ngroups) table_group<TILE, WEAK>(data, len, offsets, sizes, nblocks, digests, status, weak, order, g, tile);
}

// The length class of a block for sha1_table_kernel's `order` (sf_sort.hip's
// counting sort): the block's compression count on a log scale with `mbits`
// mantissa bits (classes 6.25 % wide with 4 bits, exact below 16; the key is
// clamped to kmax = 255, so every block of >= 2^16 compressions shares the top
// class).  A class holds many blocks, so a wave's 64 blocks (consecutive in
// the stable sort: list order within a class) lie close together in memory;
// an exact-count key spreads them over the whole buffer (every nch value is
// rare), and 64 lanes streaming from 64 far-apart places run memory-bound:
// 4 KiB blocks in a shuffled order hashed at 1200 GiB/s against 2857 in order
// (scripts/ragged_probe.py).
__device__ __forceinline__ uint16_t length_class(uint32_t nch, uint32_t mbits) {
  if (nch < (1u << mbits)) return (uint16_t)nch;
  const uint32_t e = 31u - (uint32_t)__builtin_clz(nch);  // floor(log2), >= mbits
  return (uint16_t)((e << mbits) + ((nch >> (e - mbits)) & ((1u << mbits) - 1u)));  // < 32 << mbits
}

// Wire emission of the signature table as the reference's FILE_BLOCK
// messages (src/sync/ssh/proto.rs:162-166): "FILE_BLOCK\n" + 20 raw digest
// bytes + "\n" + decimal size + "\n".  Fixed tiling: every block is
// block_size bytes except the last (last_size), so message i starts at
// i * (33 + digits(block_size)).  One thread per message, byte stores.
__device__ __forceinline__ uint32_t dec_digits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) { v /= 10; ++d; }
  return d;
}

#ifndef SF_STREAM_TU
__global__ void __launch_bounds__(256)
wire_file_blocks_kernel(const uint8_t* __restrict__ digests, uint64_t n, uint32_t block_size, uint32_t last_size,
                        uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t db = dec_digits(block_size);
  const uint64_t msg = 33 + db;  // 11 + 20 + 1 + digits + 1
  uint8_t* o = out + i * msg;
  const char tag[11] = {'F', 'I', 'L', 'E', '_', 'B', 'L', 'O', 'C', 'K', '\n'};
#pragma unroll
  for (int k = 0; k < 11; ++k) o[k] = (uint8_t)tag[k];
  const uint8_t* d = digests + i * 20;
#pragma unroll
  for (int k = 0; k < 20; ++k) o[11 + k] = d[k];
  o[31] = '\n';
  uint32_t v = (i + 1 == n) ? last_size : block_size;
  const uint32_t nd = dec_digits(v);
  for (int k = (int)nd - 1; k >= 0; --k) { o[32 + k] = (uint8_t)('0' + v % 10); v /= 10; }
  o[32 + nd] = '\n';
}
#endif

// splitmix64 byte stream: word i = mix(seed + (i+1)*GAMMA),
// little-endian; writes bytes [start, start+len) of the stream.
__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

#ifndef SF_STREAM_TU
__global__ void __launch_bounds__(256)
fill_splitmix_kernel(uint8_t* __restrict__ out, uint64_t len, uint64_t seed, uint64_t start) {
  // Fast path: whole 16-B groups of 2 aligned stream words.
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  if ((start & 15u) == 0 && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    const uint64_t nvec = len / 16;
    const uint64_t w0 = start / 8;
    for (uint64_t v = tid; v < nvec; v += stride) {
      const uint64_t a = splitmix_word(seed, w0 + 2 * v), b = splitmix_word(seed, w0 + 2 * v + 1);
      reinterpret_cast<ulonglong2*>(out)[v] = make_ulonglong2(a, b);
    }
    for (uint64_t p = nvec * 16 + tid; p < len; p += stride) {
      const uint64_t sp = start + p;
      out[p] = (uint8_t)(splitmix_word(seed, sp >> 3) >> (8 * (sp & 7)));
    }
  } else {
    for (uint64_t p = tid; p < len; p += stride) {
      const uint64_t sp = start + p;
      out[p] = (uint8_t)(splitmix_word(seed, sp >> 3) >> (8 * (sp & 7)));
    }
  }
}
#endif


}  // namespace sf
