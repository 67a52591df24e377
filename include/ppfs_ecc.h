/*
 * ppfs_ecc.h -- C ABI of the MI355X (gfx950) per-block ECC engine.
 *
 * This is the drop-in boundary underneath PPFS's IBlockDevice layer
 * (reference: lib/blockdevice/include/ppfs/blockdevice/iblock_device.hpp:34-97).
 * Each entry point replaces the per-block arithmetic of one reference codec with a batch
 * of blocks processed by hand-written HIP kernels:
 *
 *   ppfs_ecc_encode  <- ReedSolomonBlockDevice::_encodeBlock   rs_block_device.cpp:95-117
 *                       CrcBlockDevice::_calculateAndWrite     crc_block_device.cpp:37-67
 *                       HammingBlockDevice::_encodeData        hamming_block_device.cpp:76-109
 *                       ParityBlockDevice::writeBlock (parity) parity_block_device.cpp:49-54
 *   ppfs_ecc_decode  <- ReedSolomonBlockDevice::_fixBlockAndExtract  rs_block_device.cpp:119-183
 *                       CrcBlockDevice::_readAndCheckRaw             crc_block_device.cpp:12-35
 *                       HammingBlockDevice::_readAndFixBlock/_extractData hamming_block_device.cpp:21-74
 *                       ParityBlockDevice::_checkParity              parity_block_device.cpp:90-97
 *   ppfs_ecc_write   <- IBlockDevice::writeBlock of a full payload at offset 0
 *                       (read-modify-write: check/fix the old block, then encode)
 *   ppfs_ecc_create  <- PpFS::_createAppropriateBlockDevice   lib/filesystem/src/ppfs.cpp:35-70
 *
 * Conventions
 *   - Plain pointers and sizes only; no exceptions cross the ABI.  Return 0 on success or a
 *     negative errno-style code.
 *   - Blocks are packed: raw block i at raw + i*raw_block_size, payload i at
 *     data + i*data_size (the on-disk image layout: IDisk address = index * rawBlockSize()).
 *   - *_device functions take device pointers and a hipStream_t passed as void* (NULL =
 *     the null stream); they enqueue work and return without synchronising.
 *   - *_host functions take host pointers, stage through pinned buffers with overlapped
 *     H2D / kernel / D2H, and return after the results are in host memory.
 *   - Per-block status bytes use FsError values (lib/common/include/ppfs/common/types.hpp):
 *       PPFS_ECC_OK (0), PPFS_ECC_CORRECTED (1: the reference writes the block back and logs
 *       an ErrorCorrectionEvent), PPFS_ECC_CORRECTION_ERROR (5 = BlockDevice_CorrectionError).
 *   - One context per (host thread, GPU); a context is not internally locked.
 */
#ifndef PPFS_ECC_H
#define PPFS_ECC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ECCType (lib/blockdevice/include/ppfs/blockdevice/ecc_type.hpp:8-14) */
enum ppfs_ecc_type {
    PPFS_ECC_NONE = 0,
    PPFS_ECC_CRC = 1,
    PPFS_ECC_HAMMING = 2,
    PPFS_ECC_PARITY = 3,
    PPFS_ECC_REED_SOLOMON = 4
};

enum ppfs_ecc_status {
    PPFS_ECC_OK = 0,
    PPFS_ECC_CORRECTED = 1,
    PPFS_ECC_CORRECTION_ERROR = 5
};

/* Error codes returned by the entry points. */
#define PPFS_ECC_EINVAL (-22)
#define PPFS_ECC_ENOMEM (-12)
#define PPFS_ECC_EHIP (-5)
#define PPFS_ECC_ENOTSUP (-95)

/* Parameters persisted in the SuperBlock (super_block.hpp:20-23) / FsConfig (types.hpp:47-70). */
typedef struct ppfs_ecc_params {
    uint32_t ecc_type;             /* enum ppfs_ecc_type */
    uint32_t block_size;           /* FS block size in bytes (<= 4096, MAX_BLOCK_SIZE) */
    uint32_t rs_correctable_bytes; /* Reed-Solomon t (clamped to min(block,255)/2 like the reference) */
    uint32_t reserved;
    uint64_t crc_polynomial;       /* CRC polynomial in EXPLICIT form (CrcPolynomial::MsgExplicit) */
} ppfs_ecc_params;

typedef struct ppfs_ecc_ctx ppfs_ecc_ctx;

/* Convert a config-file ("implicit +1") CRC polynomial to the explicit form:
 * CrcPolynomial::MsgImplicit, crc_polynomial.cpp:41-54.  */
uint64_t ppfs_ecc_crc_implicit_to_explicit(uint64_t implicit_poly);

/* Create a codec context on HIP device `device`.  Validates params with the reference's
 * clamping rules; builds and uploads the codec tables.  */
int ppfs_ecc_create(const ppfs_ecc_params* params, int device, ppfs_ecc_ctx** out);
void ppfs_ecc_destroy(ppfs_ecc_ctx* ctx);

/* IBlockDevice::rawBlockSize() / dataSize() of the equivalent reference device. */
size_t ppfs_ecc_raw_block_size(const ppfs_ecc_ctx* ctx);
size_t ppfs_ecc_data_size(const ppfs_ecc_ctx* ctx);

/* Short human-readable name of the kernel path the context dispatches to (for logs/tests). */
const char* ppfs_ecc_kernel_name(const ppfs_ecc_ctx* ctx);
/* The kernel path a device call of ctx on `stream` takes: as ppfs_ecc_kernel_name, except for
 * RS 2t <= 8 and 2t = 32, whose ticket-counter kernels need one of the context's 16 per-stream
 * counter sets: a 17th distinct stream, and any stream capturing a hipGraph, get the static-walk
 * kernels ("rs255-wg-seg4-lds" / "rs255-bs-byte-lds-static").  Engine extension, no reference
 * counterpart. */
const char* ppfs_ecc_stream_kernel_name(ppfs_ecc_ctx* ctx, void* stream);

/*
 * Encode nblocks full payloads.  raw is read-modify-write: bits the codec does not define
 * (CRC unused tail bits when degree % 8 != 0, Hamming bits after the last data bit) keep
 * raw's previous contents exactly as the reference's writeBlock keeps the old block's.
 */
int ppfs_ecc_encode_device(ppfs_ecc_ctx* ctx, const uint8_t* d_data, uint8_t* d_raw, size_t nblocks,
    void* stream);

/*
 * Decode / check nblocks raw blocks.
 *   d_data    (may be NULL) receives the payloads (undefined for blocks with status 5).
 *   d_status  (may be NULL) receives one status byte per block.
 *   write_back != 0 applies the reference's write-back to d_raw in place (RS: the corrected
 *             bytes of the codeword; Hamming: the one flipped byte).
 *   d_spill   (RS only, may be NULL; meaningful only when rawBlockSize() < 255): per block
 *             (256 - rawBlockSize()) bytes: [0] = bytes the reference's write-back writes
 *             past the end of the block, [1..] = those bytes.  Blocks are decoded
 *             independently; a spill is reported, never applied to the neighbouring block.
 */
int ppfs_ecc_decode_device(ppfs_ecc_ctx* ctx, uint8_t* d_raw, uint8_t* d_data, uint8_t* d_status,
    size_t nblocks, int write_back, uint8_t* d_spill, void* stream);

/*
 * writeBlock(full payload, {i, 0}) for nblocks blocks: check/fix the old block held in
 * d_raw, then encode d_data into it.  d_status (may be NULL): 0, 1 (old block corrected and
 * logged), 5 (old block failed its check: the reference returns CorrectionError and leaves
 * the block untouched -- CRC, parity, uncorrectable Hamming).
 */
int ppfs_ecc_write_device(ppfs_ecc_ctx* ctx, const uint8_t* d_data, uint8_t* d_raw, uint8_t* d_status,
    size_t nblocks, void* stream);

/* Host-memory variants (chunked, H2D/kernel/D2H overlapped on two streams).  Pageable caller
 * buffers go through the context's pinned staging buffers (one CPU copy each way); when every
 * caller buffer of the call is page-locked (hipHostMalloc, or ppfs_ecc_host_register below) the
 * chunks are DMA'd straight between the caller's memory and the device. */
int ppfs_ecc_encode_host(ppfs_ecc_ctx* ctx, const uint8_t* data, uint8_t* raw, size_t nblocks);
int ppfs_ecc_decode_host(ppfs_ecc_ctx* ctx, uint8_t* raw, uint8_t* data, uint8_t* status, size_t nblocks,
    int write_back, uint8_t* spill);
int ppfs_ecc_write_host(ppfs_ecc_ctx* ctx, const uint8_t* data, uint8_t* raw, uint8_t* status,
    size_t nblocks);
/* Blocks per staging chunk of the host calls above (16 MiB of codewords, a multiple of 1 Ki).  A
 * decode with write-back of RS(255, k) or Hamming returns the bytes its write-back changed as a
 * patch list that the host writes into raw; other codecs return the changed codewords whole.
 * Engine extension, no reference counterpart. */
size_t ppfs_ecc_host_chunk_blocks(ppfs_ecc_ctx* ctx);

/*
 * Whole-image scrub: the disk-image effect of readBlock(i, 0, dataSize()) for
 * i = 0 .. nblocks-1 in index order, without the payloads -- RS writes back the corrected
 * codeword (rs_block_device.cpp:175-180), Hamming the flipped byte (hamming_block_device.cpp:41-51),
 * CRC and parity only check (crc_block_device.cpp:12-35, parity_block_device.cpp:90-97).
 *   image        packed raw blocks from block 0; image_bytes >= nblocks * rawBlockSize() is the
 *                extent a write-back may touch (a shortened RS code, n < 255, can write up to
 *                255 - n bytes past a block end: into the next blocks, which are then scrubbed as
 *                modified, as the sequential reference reads them; a write-back that would pass
 *                image_bytes is rejected whole, like HeapDisk::write, heap_disk.cpp:21-27).
 *   status       (may be NULL) one status byte per block.
 *   counts       (host form, may be NULL) [blocks ok, blocks corrected, blocks failed].
 * The device form enqueues on `stream`; with n < 255 it synchronises between runs of blocks.
 */
int ppfs_ecc_scrub_host(ppfs_ecc_ctx* ctx, uint8_t* image, size_t image_bytes, size_t nblocks, uint8_t* status,
    size_t* counts);
int ppfs_ecc_scrub_device(ppfs_ecc_ctx* ctx, uint8_t* d_image, size_t image_bytes, size_t nblocks,
    uint8_t* d_status, void* stream);

/*
 * 2-of-3 bitwise majority of nrec replicated records of rec_bytes each, replacing
 * SuperBlockManager::_performBitVoting (lib/super_block_manager/src/super_block_manager.cpp:133-165):
 *   out[i] = majority(a[i], b[i], c[i]) bit by bit;
 *   damaged (may be NULL) per record: bit k set when copy k+1 differs from the majority
 *   (the reference's damaged1/2/3).
 * The host form runs on HIP device `device` and returns when the outputs are in host memory.
 */
int ppfs_vote3_device(const uint8_t* d_a, const uint8_t* d_b, const uint8_t* d_c, uint8_t* d_out, size_t rec_bytes,
    size_t nrec, uint32_t* d_damaged, void* stream);
int ppfs_vote3_host(int device, const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out, size_t rec_bytes,
    size_t nrec, uint32_t* damaged);

/*
 * Device-to-device copy of `bytes` (any alignment) on `stream`: the measurement reference for
 * the HBM roofline ("also measure a device-to-device copy kernel on the box and report
 * both fractions").  Not a reference interface: full-grid 16-byte copy, see DESIGN.md section 5.
 */
int ppfs_copy_device(void* d_dst, const void* d_src, size_t bytes, void* stream);

/*
 * Fault injection, one byte per block: block b of the raw image (stride bytes per block) gets
 * byte pos[b] set to val[b] (mode 0) or XORed with val[b] (mode 1); pos[b] >= stride leaves the
 * block alone.  Positions are one byte each, so only the first 256 bytes of a block are
 * reachable.  The device-side counterpart of the reference's bit flipper
 * (usage_simulator/simulation/src/bit_flipper.cpp), which is out of scope as a simulator: this
 * entry exists for bench.py's corrupt-then-decode step and the tests.  Not a reference interface.
 */
int ppfs_inject_device(uint8_t* d_raw, size_t stride, size_t nblocks, const uint8_t* d_pos, const uint8_t* d_val,
    int mode, void* stream);

/*
 * Page-lock / release a caller buffer (hipHostRegister), e.g. the host mirror of a disk image
 * (replacing FileDisk's seekp + fstream I/O, lib/disk/src/file_disk.cpp:56-101,
 * by an mmap'd or resident image the *_host calls then DMA directly).
 */
int ppfs_ecc_host_register(void* ptr, size_t bytes);
int ppfs_ecc_host_unregister(void* ptr);
/* Ranges registered through ppfs_ecc_host_register and not yet unregistered: their number (and
 * their total bytes in *bytes when bytes is non-null).  Diagnostics: tests assert that no range
 * outlives the test that registered it.  Engine extension, no reference counterpart. */
long long ppfs_ecc_host_registered(size_t* bytes);

/*
 * Multi-GPU host path: a group of contexts, one per listed HIP device (a device may
 * repeat), over which the *_host calls shard a batch into contiguous block ranges -- shard g =
 * blocks [g*N/G, (g+1)*N/G), one contiguous range of the packed image -- each run by its own host
 * thread on its context's streams and pinned staging.  Blocks are independent codewords: no data
 * moves between devices and no collective runs; the call returns when every shard's results are in
 * host memory, with the first failing shard's error.  Status / spill are split like the blocks.
 * (Reference: the caller side of IBlockDevice, file_io.cpp:12-104, issues the same per-block work
 * serially on one CPU thread.)
 */
typedef struct ppfs_ecc_group ppfs_ecc_group;
int ppfs_ecc_group_create(const ppfs_ecc_params* params, const int* devices, int ndevices, ppfs_ecc_group** out);
void ppfs_ecc_group_destroy(ppfs_ecc_group* group);
int ppfs_ecc_group_size(const ppfs_ecc_group* group);
ppfs_ecc_ctx* ppfs_ecc_group_ctx(ppfs_ecc_group* group, int index);
int ppfs_ecc_group_encode_host(ppfs_ecc_group* group, const uint8_t* data, uint8_t* raw, size_t nblocks);
int ppfs_ecc_group_decode_host(ppfs_ecc_group* group, uint8_t* raw, uint8_t* data, uint8_t* status, size_t nblocks,
    int write_back, uint8_t* spill);
int ppfs_ecc_group_write_host(ppfs_ecc_group* group, const uint8_t* data, uint8_t* raw, uint8_t* status,
    size_t nblocks);

/* Kernel timing hook (bench.py's roofline, tools): the next RS kernel the calling thread launches
 * through any context records start_event / stop_event (hipEvent_t, created by the caller with
 * timing enabled) from its own dispatch packet (hipExtLaunchKernel) -- the kernel's execution time
 * as rocprofv3 measures it, without the launch gap that events recorded on the stream around the
 * call include.  The hook disarms after one launch; (NULL, NULL) disarms it.  -EINVAL if only one
 * event is given.  Engine extension, no reference counterpart. */
int ppfs_ecc_time_next_launch(void* start_event, void* stop_event);

/* Last HIP error string recorded by this thread (diagnostics). */
const char* ppfs_ecc_last_error(void);

/* Diagnostics of PPFS_ECC_DEBUG builds (csrc/dbg.hpp): the number of out-of-bounds global
 * accesses the kernels detected (and skipped) so far; -1 in normal builds.  Engine extension,
 * no reference counterpart. */
long long ppfs_ecc_debug_faults(void);
/* PPFS_ECC_DEBUG builds: launches one deliberately out-of-range row gather and returns how many
 * accesses the kernel reported (and skipped), >= 1 when the checks work; -1 in normal builds. */
long long ppfs_ecc_debug_selftest(void);
/* PPFS_ECC_DEBUG builds: copies the engine refused because an end was not page-locked host memory /
 * device memory over its whole range (every hipMemcpy the library issues is checked first);
 * -1 in normal builds. */
long long ppfs_ecc_debug_dma_rejects(void);
/* PPFS_ECC_DEBUG builds: positive control of those checks (a pageable source and a device range past
 * its allocation must both be refused): 1 when they are, 0 when not, -1 in normal builds. */
long long ppfs_ecc_debug_dma_selftest(void);

#ifdef __cplusplus
}
#endif

#endif /* PPFS_ECC_H */
