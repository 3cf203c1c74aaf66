"""juicefs_amd -- MI355X block-transform engine for the JuiceFS per-block path.

AES-256-GCM / ChaCha20-Poly1305 Seal/Open (pkg/object/encrypt.go) fused with
CRC32C 32 KiB segment checksums (pkg/chunk/disk_cache.go), as hand-written HIP
kernels for gfx950 behind a C-ABI (include/jfsx.h, libjfsx.so).

Modules:
  engine   -- ctypes binding of libjfsx.so (no CPU fallback)
  encrypt  -- object.Encryptor mirror: NewDataEncryptor / Encrypt / Decrypt,
              RSA-OAEP key wrapping, the encrypted object-store wrapper
  chunk    -- checksum() and cacheFile.ReadAt (none/full/shrink/extend)
"""
from .engine import (AES256GCM, CHACHA20P1305, CRC_GEN, CRC_NONE, CRC_VERIFY, MEM_DEVICE, MEM_HOST,  # noqa: F401
                     ChecksumError, DeviceBuffer, Engine, EngineError, load_library)

__version__ = "0.1.0"
