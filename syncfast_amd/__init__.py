"""syncfast_amd -- MI355X-native block-signature indexing for syncfast.

The hot path of syncfast's ``Index::index_file`` (/root/reference/src/index.rs:
610-659) -- SHA-1 of every block plus the per-file ``blocks_hash`` -- as
hand-written gfx950 HIP kernels behind a C-ABI (include/syncfast_amd.h).

Modules
  device  -- HBM-resident entry points over torch tensors (the hot path)
  host    -- host-memory / file entry points (end-to-end, incl. H2D/D2H)
  digest  -- HashDigest, the signature value type (src/lib.rs:72-145)
  index   -- Index, the reference's library API on SQLite (src/index.rs)
  timestamp -- files.modified as chrono's DateTime<Utc> (src/index.rs:176-218)
  shard   -- multi-GPU sharding + RCCL gather of the signature table, and one
             file on disk indexed by every rank
  wire    -- FILE_BLOCK / FILE_ENTRY framing (src/sync/ssh/proto.rs) and the
             device-built FILE_BLOCK run
"""
from ._lib import (HASH_DIGEST_LEN, LIB_PATH, MAX_BLOCK_SIZE, SfError, device_count,  # noqa: F401
                   lib)

__version__ = "0.1.0"
