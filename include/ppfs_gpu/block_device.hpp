#pragma once
/*
 * ppfs_gpu/block_device.hpp -- C++17 host mirror of PPFS's block-device layer, backed by the
 * MI355X ECC engine (include/ppfs_ecc.h).  Header-only; link with libppfs_ecc.so.
 *
 * Same class names, constructor arguments, return conventions and error behaviour as the
 * reference, so PPFS code (FileIO, Bitmap, InodeManager, bench_blockdevice) can hold these
 * objects where it holds the reference's:
 *
 *   IBlockDevice               lib/blockdevice/include/ppfs/blockdevice/iblock_device.hpp:34-97
 *   DataLocation               iblock_device.hpp:14-20
 *   ReedSolomonBlockDevice     rs_block_device.hpp:20-80,  src/rs_block_device.cpp:9-93
 *   CrcBlockDevice             crc_block_device.hpp,       src/crc_block_device.cpp:12-134
 *   HammingBlockDevice         hamming_block_device.hpp,   src/hamming_block_device.cpp:11-172
 *   ParityBlockDevice          parity_block_device.hpp,    src/parity_block_device.cpp:9-97
 *   RawBlockDevice             raw_block_device.hpp,       src/raw_block_device.cpp
 *   CrcPolynomial              lib/ecc_helpers/include/ppfs/ecc_helpers/crc_polynomial.hpp
 *   IDisk / StackDisk          lib/disk/include/ppfs/disk/idisk.hpp:9-19, stack_disk.hpp:9-44
 *   static_vector              lib/common/include/ppfs/common/static_vector.hpp:11-100
 *   FsError                    lib/common/include/ppfs/common/types.hpp:11-80 (same order/values)
 *
 * The reference is C++23 (std::expected); this image's libstdc++ has no <expected>, so
 * ppfs_gpu::expected / unexpected carry the same interface (has_value, value, error,
 * operator bool).  Inside PPFS proper, alias them to std:: and drop the copies here.
 *
 * All codec arithmetic (RS encode / syndromes / Berlekamp-Massey / Chien / Forney, CRC,
 * Hamming SECDED, parity) runs in the HIP kernels behind the C ABI.  This layer moves bytes
 * between the disk and the engine and reproduces the reference's read-modify-write,
 * write-back and logging order.  There is no CPU fallback: every engine error (including a
 * device whose engine could not be created: no GPU, bad parameters) is reported as
 * FsError::Disk_IOError, with the ABI's message on stderr; nothing throws or aborts.
 *
 * Extension: readBlocks / writeBlocks run a contiguous range of whole blocks
 * through ONE engine call; results, disk contents and log are those of the per-block loop.
 */
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "ppfs_ecc.h"

#define MAX_BLOCK_SIZE 4096
#define MAX_RS_BLOCK_SIZE 255

namespace ppfs_gpu {

typedef std::uint32_t block_index_t;

enum class FsError : uint8_t {
    Bitmap_IndexOutOfRange,
    Bitmap_NotFound,
    BlockManager_AlreadyTaken,
    BlockManager_AlreadyFree,
    BlockManager_NoMoreFreeBlocks,
    BlockDevice_CorrectionError, // = 5
    DirectoryManager_NameTaken,
    DirectoryManager_NotFound,
    DirectoryManager_InvalidRequest,
    Disk_OutOfBounds, // = 9
    Disk_InvalidRequest, // = 10
    Disk_IOError, // = 11
    FileIO_OutOfBounds,
    FileIO_InternalError,
    FileIO_InvalidRequest,
    PpFS_DiskNotFormatted,
    PpFS_InvalidRequest,
    PpFS_NotInitialized,
    PpFS_InvalidPath,
    PpFS_NotFound,
    PpFS_FileInUse,
    PpFS_DirectoryNotEmpty,
    PpFS_OutOfBounds,
    PpFS_OpenFilesTableFull,
    PpFS_AlreadyOpen,
    InodeManager_AlreadyTaken,
    InodeManager_NotFound,
    InodeManager_AlreadyFree,
    InodeManager_NoMoreFreeInodes,
    Mutex_InitFailed,
    Mutex_LockFailed,
    Mutex_UnlockFailed,
    Mutex_NotInitialized,
    Mutex_AlreadyInitialized,
    Mutex_InternalError,
    SuperBlockManager_InvalidRequest,
    StaticVector_AllocationError,
    NotImplemented,
    Config_IOError,
    Config_SyntaxError,
    Config_InvalidValue,
    Config_MissingField,
    Config_UnknownKey
};
static_assert((int)FsError::BlockDevice_CorrectionError == PPFS_ECC_CORRECTION_ERROR, "status 5");

// ------------------------------------------------------------------------------------------
// std::expected<T, E> subset
// ------------------------------------------------------------------------------------------
template <class E> struct unexpected_t {
    E e;
};
template <class E> unexpected_t<E> unexpected(E e) { return { e }; }

template <class T, class E = FsError> class expected {
public:
    expected(T v)
        : _ok(true)
        , _v(std::move(v))
    {
    }
    expected(unexpected_t<E> u)
        : _ok(false)
        , _e(u.e)
    {
    }
    bool has_value() const { return _ok; }
    explicit operator bool() const { return _ok; }
    const T& value() const
    {
        if (!_ok) {
            std::fprintf(stderr, "ppfs_gpu::expected: bad access (error %d)\n", (int)_e);
            std::abort();
        }
        return _v;
    }
    const T& operator*() const { return _v; }
    E error() const { return _e; }

private:
    bool _ok;
    T _v {};
    E _e {};
};

template <class E> class expected<void, E> {
public:
    expected()
        : _ok(true)
    {
    }
    expected(unexpected_t<E> u)
        : _ok(false)
        , _e(u.e)
    {
    }
    bool has_value() const { return _ok; }
    explicit operator bool() const { return _ok; }
    void value() const
    {
        if (!_ok) {
            std::fprintf(stderr, "ppfs_gpu::expected: bad access (error %d)\n", (int)_e);
            std::abort();
        }
    }
    E error() const { return _e; }

private:
    bool _ok;
    E _e {};
};

// ------------------------------------------------------------------------------------------
// static_vector: non-owning view with a capacity (static_vector.hpp semantics)
// ------------------------------------------------------------------------------------------
template <typename T> class static_vector {
    static_assert(std::is_trivially_copyable<T>::value, "static_vector supports only trivially copyable types");

public:
    static_vector() = default;
    static_vector(T* buffer, std::size_t capacity, std::size_t size = 0)
        : _buffer(buffer)
        , _capacity(capacity)
        , _size(std::min(size, capacity))
    {
    }
    expected<void> push_back(const T& v)
    {
        if (_size >= _capacity)
            return unexpected(FsError::StaticVector_AllocationError);
        _buffer[_size++] = v;
        return {};
    }
    T& operator[](std::size_t i) { return _buffer[i]; }
    const T& operator[](std::size_t i) const { return _buffer[i]; }
    std::size_t size() const { return _size; }
    std::size_t capacity() const { return _capacity; }
    bool empty() const { return _size == 0; }
    T* begin() { return _buffer; }
    T* end() { return _buffer + _size; }
    const T* begin() const { return _buffer; }
    const T* end() const { return _buffer + _size; }
    T* data() { return _buffer; }
    const T* data() const { return _buffer; }
    expected<void> resize(std::size_t n)
    {
        if (n > _capacity)
            return unexpected(FsError::StaticVector_AllocationError);
        _size = n;
        return {};
    }
    expected<void> assign(std::initializer_list<T> init)
    {
        if (init.size() > _capacity)
            return unexpected(FsError::StaticVector_AllocationError);
        std::memcpy(_buffer, init.begin(), init.size() * sizeof(T));
        _size = init.size();
        return {};
    }

private:
    T* _buffer = nullptr;
    std::size_t _capacity = 0;
    std::size_t _size = 0;
};

struct DataLocation {
    int block_index = 0;
    size_t offset = 0;
    DataLocation(int b, size_t o)
        : block_index(b)
        , offset(o)
    {
    }
    DataLocation() = default;
};

// ------------------------------------------------------------------------------------------
// Disks
// ------------------------------------------------------------------------------------------
struct IDisk {
    virtual ~IDisk() = default;
    virtual expected<void> read(size_t address, size_t size, static_vector<uint8_t>& data) = 0;
    virtual expected<size_t> write(size_t address, const static_vector<uint8_t>& data) = 0;
    virtual size_t size() = 0;
    // Extension: a disk whose whole image is addressable host memory (size() bytes, writes
    // through it are the disk's writes).  The batch calls of the engine devices then run the
    // engine on the image in place -- no copy into and out of a staging vector.  nullptr: no.
    virtual uint8_t* mapped() { return nullptr; }
};

// In-memory disk with StackDisk's semantics (stack_disk.hpp:19-44: out-of-range accesses
// fail whole; read checks bounds, then capacity).  Storage is heap-allocated.
template <size_t power = 22> class StackDisk : public IDisk {
public:
    StackDisk()
        : _data(size_t(1) << power, 0)
    {
    }
    size_t size() override { return _data.size(); }
    expected<void> read(size_t address, size_t size, static_vector<uint8_t>& data) override
    {
        if (address + size > _data.size())
            return unexpected(FsError::Disk_OutOfBounds);
        if (data.capacity() < size)
            return unexpected(FsError::Disk_InvalidRequest);
        data.resize(size);
        std::memcpy(data.data(), _data.data() + address, size);
        return {};
    }
    expected<size_t> write(size_t address, const static_vector<uint8_t>& data) override
    {
        if (address + data.size() > _data.size())
            return unexpected(FsError::Disk_OutOfBounds);
        std::memcpy(_data.data() + address, data.data(), data.size());
        return data.size();
    }
    uint8_t* image() { return _data.data(); }
    uint8_t* mapped() override { return _data.data(); }

private:
    std::vector<uint8_t> _data;
};

// File-backed disk with FileDisk's interface and checks (file_disk.hpp, file_disk.cpp:8-101:
// open an existing file / create a zero-filled one of a fixed size; read checks open, bounds,
// then capacity; write checks open and bounds), over a shared mmap of the file instead of
// fstream seek + read / write.  The mapping is page-locked for the engine when the
// HIP runtime allows it (ppfs_ecc_host_register; a file mapping it cannot pin stays pageable), so
// the batch calls DMA straight between the page cache and HBM.
class MappedFileDisk : public IDisk {
public:
    MappedFileDisk() = default;
    ~MappedFileDisk() override { close(); }
    MappedFileDisk(const MappedFileDisk&) = delete;
    MappedFileDisk& operator=(const MappedFileDisk&) = delete;

    expected<void> open(const std::string& path)
    {
        close();
        const int fd = ::open(path.c_str(), O_RDWR);
        if (fd < 0)
            return unexpected(FsError::Disk_IOError);
        struct stat st;
        if (::fstat(fd, &st) != 0) {
            ::close(fd);
            return unexpected(FsError::Disk_IOError);
        }
        _size = (size_t)st.st_size;
        if (_size) {
            void* m = ::mmap(nullptr, _size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) {
                ::close(fd);
                _size = 0;
                return unexpected(FsError::Disk_IOError);
            }
            _map = (uint8_t*)m;
            _pinned = ppfs_ecc_host_register(_map, _size) == 0;
        }
        _fd = fd;
        return {};
    }
    expected<void> create(const std::string& path, size_t size)
    {
        if (_fd >= 0)
            return unexpected(FsError::Disk_InvalidRequest); // file_disk.cpp:37-38
        const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
        if (fd < 0)
            return unexpected(FsError::Disk_IOError);
        const bool ok = ::ftruncate(fd, (off_t)size) == 0;
        ::close(fd);
        if (!ok)
            return unexpected(FsError::Disk_IOError);
        return open(path);
    }
    void close()
    {
        if (_map) {
            if (_pinned)
                (void)ppfs_ecc_host_unregister(_map);
            ::msync(_map, _size, MS_SYNC);
            ::munmap(_map, _size);
        }
        if (_fd >= 0)
            ::close(_fd);
        _map = nullptr;
        _fd = -1;
        _size = 0;
        _pinned = false;
    }
    size_t size() override { return _size; }
    bool pinned() const { return _pinned; }
    uint8_t* mapped() override { return _map; }
    expected<void> read(size_t address, size_t size, static_vector<uint8_t>& data) override
    {
        if (_fd < 0)
            return unexpected(FsError::Disk_IOError);
        if (address + size > _size)
            return unexpected(FsError::Disk_OutOfBounds);
        if (data.capacity() < size)
            return unexpected(FsError::Disk_InvalidRequest);
        data.resize(size);
        if (size)
            std::memcpy(data.data(), _map + address, size);
        return {};
    }
    expected<size_t> write(size_t address, const static_vector<uint8_t>& data) override
    {
        if (_fd < 0)
            return unexpected(FsError::Disk_IOError);
        if (address + data.size() > _size)
            return unexpected(FsError::Disk_OutOfBounds);
        if (data.size())
            std::memcpy(_map + address, data.data(), data.size());
        return data.size();
    }

private:
    int _fd = -1;
    uint8_t* _map = nullptr;
    size_t _size = 0;
    bool _pinned = false;
};

// ------------------------------------------------------------------------------------------
// Logger: block devices emit only ErrorCorrectionEvent (rs:171-173, hamming:53-57)
// ------------------------------------------------------------------------------------------
struct ErrorCorrectionEvent {
    std::string codec;
    block_index_t block_index;
    ErrorCorrectionEvent(std::string c, block_index_t b)
        : codec(std::move(c))
        , block_index(b)
    {
    }
};

class Logger {
public:
    virtual ~Logger() = default;
    virtual void logEvent(const ErrorCorrectionEvent& e) { events.push_back(e); }
    std::vector<ErrorCorrectionEvent> events;
};

// ------------------------------------------------------------------------------------------
// CrcPolynomial (crc_polynomial.cpp:7-54)
// ------------------------------------------------------------------------------------------
class CrcPolynomial {
public:
    static CrcPolynomial MsgExplicit(uint64_t p) { return CrcPolynomial(p); }
    static CrcPolynomial MsgImplicit(uint64_t p) { return CrcPolynomial(ppfs_ecc_crc_implicit_to_explicit(p)); }
    uint64_t getExplicitPolynomial() const { return _p; }
    uint64_t getImplicitPolynomial() const { return _p >> 1; }
    int getDegree() const
    {
        int n = -1;
        for (uint64_t v = _p; v; v >>= 1)
            ++n;
        return n;
    }

private:
    explicit CrcPolynomial(uint64_t p)
        : _p(p)
    {
    }
    uint64_t _p;
};

// ------------------------------------------------------------------------------------------
// Engine handle (one codec context on one GPU)
// ------------------------------------------------------------------------------------------
class EccEngine {
public:
    EccEngine(uint32_t type, uint32_t block_size, uint32_t t, uint64_t poly, int device)
    {
        ppfs_ecc_params p {};
        p.ecc_type = type;
        p.block_size = block_size;
        p.rs_correctable_bytes = t;
        p.crc_polynomial = poly;
        // the reference's constructors cannot fail: a device whose engine could not be created
        // (no GPU, bad parameters) reports Disk_IOError from every call instead -- no CPU fallback
        const int rc = ppfs_ecc_create(&p, device, &_ctx);
        if (rc != 0 || !_ctx) {
            std::fprintf(stderr, "ppfs_gpu: ppfs_ecc_create failed (%d): %s\n", rc, ppfs_ecc_last_error());
            _ctx = nullptr;
        }
    }
    ~EccEngine() { ppfs_ecc_destroy(_ctx); }
    EccEngine(const EccEngine&) = delete;
    EccEngine& operator=(const EccEngine&) = delete;
    size_t raw() const { return ppfs_ecc_raw_block_size(_ctx); }
    size_t data() const { return ppfs_ecc_data_size(_ctx); }
    ppfs_ecc_ctx* ctx() const { return _ctx; }
    bool valid() const { return _ctx != nullptr; }
    // An engine call's return code: 0 -> true; else the ABI's message goes to stderr and the
    // caller returns FsError::Disk_IOError (the reference's code for a failed device operation)
    static bool ok(int rc, const char* what)
    {
        if (rc != 0) {
            std::fprintf(stderr, "ppfs_gpu: %s failed (%d): %s\n", what, rc, ppfs_ecc_last_error());
            return false;
        }
        return true;
    }

private:
    ppfs_ecc_ctx* _ctx = nullptr;
};

// ------------------------------------------------------------------------------------------
// IBlockDevice
// ------------------------------------------------------------------------------------------
class IBlockDevice {
public:
    virtual ~IBlockDevice() = default;
    virtual expected<size_t> writeBlock(const static_vector<std::uint8_t>& data, DataLocation data_location) = 0;
    virtual expected<void> readBlock(DataLocation data_location, size_t bytes_to_read, static_vector<uint8_t>& data)
        = 0;
    virtual size_t rawBlockSize() const = 0;
    virtual size_t dataSize() const = 0;
    virtual size_t numOfBlocks() const = 0;
    virtual expected<void> formatBlock(unsigned int block_index) = 0;

    // Batch extension: whole blocks [first, first + count).  out: count * dataSize() bytes;
    // err (may be null): per block 0 or the FsError the per-block call returns.  The call
    // itself fails only when the range cannot be read from / written to the disk.
    virtual expected<void> readBlocks(block_index_t first, size_t count, uint8_t* out, uint8_t* err) = 0;
    virtual expected<void> writeBlocks(block_index_t first, size_t count, const uint8_t* payloads, uint8_t* err)
        = 0;

    // Whole-image scrub extension: the disk and log effect of
    // readBlock({i, 0}, dataSize()) for i in [first, first + count), in order, without the
    // payloads.  counts (may be null): blocks ok / corrected / failed; err as readBlocks.
    virtual expected<void> scrub(block_index_t first, size_t count, size_t* counts, uint8_t* err)
    {
        std::vector<uint8_t> out(count * dataSize()), e(count);
        auto r = readBlocks(first, count, out.data(), e.data());
        if (!r)
            return r;
        size_t failed = 0;
        for (uint8_t x : e)
            failed += x != 0;
        if (counts) {
            counts[0] = count - failed;
            counts[1] = 0;
            counts[2] = failed;
        }
        if (err)
            std::memcpy(err, e.data(), count);
        return {};
    }
};

namespace detail {
    inline expected<void> disk_read(IDisk& d, size_t addr, size_t n, uint8_t* dst)
    {
        static_vector<uint8_t> v(dst, n);
        return d.read(addr, n, v);
    }
    inline expected<size_t> disk_write(IDisk& d, size_t addr, const uint8_t* src, size_t n)
    {
        static_vector<uint8_t> v(const_cast<uint8_t*>(src), n, n);
        return d.write(addr, v);
    }
} // namespace detail

class RawBlockDevice : public IBlockDevice {
public:
    RawBlockDevice(size_t block_size, IDisk& disk)
        : _bs(block_size)
        , _disk(disk)
    {
    }
    size_t rawBlockSize() const override { return _bs; }
    size_t dataSize() const override { return _bs; }
    size_t numOfBlocks() const override { return _disk.size() / _bs; }
    expected<void> formatBlock(unsigned int) override { return {}; }
    expected<size_t> writeBlock(const static_vector<std::uint8_t>& data, DataLocation loc) override
    {
        const size_t to_write = std::min(data.size(), _bs - loc.offset);
        auto r = detail::disk_write(_disk, loc.block_index * _bs + loc.offset, data.data(), to_write);
        if (!r)
            return unexpected(r.error());
        return to_write;
    }
    expected<void> readBlock(DataLocation loc, size_t n, static_vector<uint8_t>& data) override
    {
        const size_t to_read = std::min(n, _bs - loc.offset);
        return _disk.read(loc.block_index * _bs + loc.offset, to_read, data);
    }
    expected<void> readBlocks(block_index_t first, size_t count, uint8_t* out, uint8_t* err) override
    {
        if (err)
            std::memset(err, 0, count);
        return detail::disk_read(_disk, (size_t)first * _bs, count * _bs, out);
    }
    expected<void> writeBlocks(block_index_t first, size_t count, const uint8_t* payloads, uint8_t* err) override
    {
        if (err)
            std::memset(err, 0, count);
        auto r = detail::disk_write(_disk, (size_t)first * _bs, payloads, count * _bs);
        if (!r)
            return unexpected(r.error());
        return {};
    }

private:
    size_t _bs;
    IDisk& _disk;
};

// Shared plumbing of the four ECC codecs: the per-block RMW path and the batched path both go
// through the engine's host entry points (pinned staging, chunked, H2D/kernel/D2H overlapped).
class EngineBlockDevice : public IBlockDevice {
public:
    size_t rawBlockSize() const override { return _raw; }
    size_t dataSize() const override { return _ds; }
    size_t numOfBlocks() const override { return _raw ? _disk.size() / _raw : 0; }

    expected<void> formatBlock(unsigned int block_index) override
    {
        // rs:15-23, hamming:164-172, parity:22-29 write an all-zero raw block; crc:124-134 an
        // all-zero payload with its CRC -- the engine's encode of a zero payload is exactly that
        std::vector<uint8_t> raw(_raw, 0), zero(_ds, 0);
        if (_type == PPFS_ECC_CRC && !EccEngine::ok(ppfs_ecc_encode_host(_eng.ctx(), zero.data(), raw.data(), 1), "encode"))
            return unexpected(FsError::Disk_IOError);
        auto r = detail::disk_write(_disk, (size_t)block_index * _raw, raw.data(), _raw);
        if (!r)
            return unexpected(r.error());
        return {};
    }

    expected<void> readBlock(DataLocation loc, size_t bytes_to_read, static_vector<uint8_t>& data) override
    {
        data.resize(0);
        if (data.capacity() < bytes_to_read)
            return unexpected(FsError::Disk_InvalidRequest);
        bytes_to_read = std::min(_ds - loc.offset, bytes_to_read);
        std::vector<uint8_t> raw(_raw), dec(_ds);
        auto rr = detail::disk_read(_disk, (size_t)loc.block_index * _raw, _raw, raw.data());
        if (!rr)
            return unexpected(rr.error());
        auto fx = check_fix(loc.block_index, raw.data(), dec.data());
        if (!fx)
            return unexpected(fx.error());
        data.resize(bytes_to_read);
        std::memcpy(data.data(), dec.data() + loc.offset, bytes_to_read);
        return {};
    }

    expected<size_t> writeBlock(const static_vector<std::uint8_t>& data, DataLocation loc) override
    {
        const size_t to_write = std::min(data.size(), _ds - loc.offset);
        std::vector<uint8_t> raw(_raw), dec(_ds);
        auto rr = detail::disk_read(_disk, (size_t)loc.block_index * _raw, _raw, raw.data());
        if (!rr)
            return unexpected(rr.error());
        auto fx = check_fix(loc.block_index, raw.data(), dec.data()); // raw: the fixed old block
        if (!fx)
            return unexpected(fx.error());
        std::memcpy(dec.data() + loc.offset, data.data(), to_write);
        // encode over the old block: CRC tail bits / Hamming unused bits keep their contents
        if (!EccEngine::ok(ppfs_ecc_encode_host(_eng.ctx(), dec.data(), raw.data(), 1), "encode"))
            return unexpected(FsError::Disk_IOError);
        auto w = detail::disk_write(_disk, (size_t)loc.block_index * _raw, raw.data(), _raw);
        if (!w)
            return unexpected(w.error());
        return to_write;
    }

    // readBlock({first + i, 0}) for i in [from, count): each block's own error (e.g.
    // Disk_OutOfBounds past the disk end) in err[i], decoded payloads (zeros on error) in out --
    // the per-block contract, for ranges the batch path cannot read in one piece
    expected<void> per_block_reads(block_index_t first, size_t from, size_t count, uint8_t* out, uint8_t* err)
    {
        for (size_t i = from; i < count; ++i) {
            static_vector<uint8_t> v(out + i * _ds, _ds, 0);
            auto r = readBlock(DataLocation((int)(first + (block_index_t)i), 0), _ds, v);
            if (!r) {
                std::memset(out + i * _ds, 0, _ds);
                if (err)
                    err[i] = (uint8_t)r.error();
            }
        }
        return {};
    }

    expected<void> readBlocks(block_index_t first, size_t count, uint8_t* out, uint8_t* err) override
    {
        if (err)
            std::memset(err, 0, count);
        if (uint8_t* img = _disk.mapped(); img && !has_spill()) {
            // in place on the disk image: the engine writes corrected codewords back into it
            // (RS: whole codeword, Hamming: the flipped byte, as the reference's write-back)
            if (((size_t)first + count) * _raw > _disk.size())
                return per_block_reads(first, 0, count, out, err); // range runs off the disk
            std::vector<uint8_t> status(count);
            if (!EccEngine::ok(ppfs_ecc_decode_host(_eng.ctx(), img + (size_t)first * _raw, out, status.data(), count,
                                   1, nullptr),
                    "decode"))
                return unexpected(FsError::Disk_IOError);
            for (size_t i = 0; i < count; ++i) {
                if (status[i] == PPFS_ECC_CORRECTION_ERROR) {
                    if (err)
                        err[i] = (uint8_t)FsError::BlockDevice_CorrectionError;
                    std::memset(out + i * _ds, 0, _ds);
                } else if (status[i] == PPFS_ECC_CORRECTED) {
                    log(first + (block_index_t)i);
                }
            }
            return {};
        }
        size_t done = 0;
        while (done < count) {
            const size_t nb = count - done;
            const block_index_t b0 = first + (block_index_t)done;
            std::vector<uint8_t> raw(nb * _raw), fixed, status(nb), spill;
            auto rr = detail::disk_read(_disk, (size_t)b0 * _raw, nb * _raw, raw.data());
            if (!rr)
                return per_block_reads(first, done, count, out, err); // range not on the disk
            fixed = raw;
            if (has_spill())
                spill.assign(nb * spill_stride(), 0);
            if (!EccEngine::ok(ppfs_ecc_decode_host(_eng.ctx(), fixed.data(), out + done * _ds, status.data(), nb,
                                 1, spill.empty() ? nullptr : spill.data()), "decode"))
                return unexpected(FsError::Disk_IOError);
            size_t i = 0;
            for (; i < nb; ++i) {
                const block_index_t b = b0 + (block_index_t)i;
                if (status[i] == PPFS_ECC_CORRECTION_ERROR) {
                    if (err)
                        err[done + i] = (uint8_t)FsError::BlockDevice_CorrectionError;
                    std::memset(out + (done + i) * _ds, 0, _ds);
                    continue;
                }
                if (status[i] != PPFS_ECC_CORRECTED)
                    continue;
                const uint8_t* sp = spill.empty() ? nullptr : spill.data() + i * spill_stride();
                auto wb = write_back(b, raw.data() + i * _raw, fixed.data() + i * _raw, sp);
                if (!wb && err)
                    err[done + i] = (uint8_t)wb.error();
                if (sp && sp[0] && i + 1 < nb) {
                    // the reference's write-back ran past this block into the next one, which
                    // the per-block loop reads afterwards: resume from there
                    ++i;
                    break;
                }
            }
            done += i;
        }
        return {};
    }

    expected<void> writeBlocks(block_index_t first, size_t count, const uint8_t* payloads, uint8_t* err) override
    {
        if (err)
            std::memset(err, 0, count);
        if (has_spill()) {
            // shortened RS codes: an old block's write-back may spill into the next block
            // before it is read; keep the per-block order exactly
            for (size_t i = 0; i < count; ++i) {
                static_vector<uint8_t> v(const_cast<uint8_t*>(payloads + i * _ds), _ds, _ds);
                auto r = writeBlock(v, DataLocation((int)(first + i), 0));
                if (!r && err)
                    err[i] = (uint8_t)r.error();
            }
            return {};
        }
        uint8_t* img = _disk.mapped();
        if (img && ((size_t)first + count) * _raw > _disk.size())
            return unexpected(FsError::Disk_OutOfBounds);
        std::vector<uint8_t> raw(img ? 0 : count * _raw), status(count);
        if (img) { // in place on the disk image
            if (!EccEngine::ok(
                ppfs_ecc_write_host(_eng.ctx(), payloads, img + (size_t)first * _raw, status.data(), count), "write"))
                return unexpected(FsError::Disk_IOError);
        } else {
            auto rr = detail::disk_read(_disk, (size_t)first * _raw, count * _raw, raw.data());
            if (!rr)
                return unexpected(rr.error());
            if (!EccEngine::ok(ppfs_ecc_write_host(_eng.ctx(), payloads, raw.data(), status.data(), count), "write"))
                return unexpected(FsError::Disk_IOError);
        }
        for (size_t i = 0; i < count; ++i) {
            if (status[i] == PPFS_ECC_CORRECTION_ERROR) {
                if (err)
                    err[i] = (uint8_t)FsError::BlockDevice_CorrectionError;
            } else if (status[i] == PPFS_ECC_CORRECTED) {
                log(first + (block_index_t)i); // the old block's write-back is overwritten below
            }
        }
        // blocks that failed their check were left untouched by the engine
        if (img)
            return {};
        auto w = detail::disk_write(_disk, (size_t)first * _raw, raw.data(), count * _raw);
        if (!w)
            return unexpected(w.error());
        return {};
    }

    // One engine call (ppfs_ecc_scrub_host) over the disk image from block `first` to the disk
    // end: the write-back of every corrected block is applied in index order, including RS
    // bytes a shortened code writes past a block end; corrected blocks are logged in order.
    expected<void> scrub(block_index_t first, size_t count, size_t* counts, uint8_t* err) override
    {
        if (err)
            std::memset(err, 0, count);
        const size_t base = (size_t)first * _raw;
        if (base + count * _raw > _disk.size())
            return unexpected(FsError::Disk_OutOfBounds);
        if (uint8_t* img = _disk.mapped()) { // in place on the disk image
            std::vector<uint8_t> status(count);
            size_t c3[3] = { 0, 0, 0 };
            if (!EccEngine::ok(
                ppfs_ecc_scrub_host(_eng.ctx(), img + base, _disk.size() - base, count, status.data(), c3), "scrub"))
                return unexpected(FsError::Disk_IOError);
            for (size_t i = 0; i < count; ++i) {
                if (status[i] == PPFS_ECC_CORRECTION_ERROR && err)
                    err[i] = (uint8_t)FsError::BlockDevice_CorrectionError;
                else if (status[i] == PPFS_ECC_CORRECTED)
                    log(first + (block_index_t)i);
            }
            if (counts)
                std::memcpy(counts, c3, sizeof c3);
            return {};
        }
        std::vector<uint8_t> image(_disk.size() - base), status(count);
        auto rr = detail::disk_read(_disk, base, image.size(), image.data());
        if (!rr)
            return unexpected(rr.error());
        const std::vector<uint8_t> before = image;
        size_t c3[3] = { 0, 0, 0 };
        if (!EccEngine::ok(ppfs_ecc_scrub_host(_eng.ctx(), image.data(), image.size(), count, status.data(), c3), "scrub"))
            return unexpected(FsError::Disk_IOError);
        for (size_t i = 0; i < count; ++i) {
            if (status[i] == PPFS_ECC_CORRECTION_ERROR && err)
                err[i] = (uint8_t)FsError::BlockDevice_CorrectionError;
            else if (status[i] == PPFS_ECC_CORRECTED)
                log(first + (block_index_t)i);
        }
        size_t lo = 0, hi = image.size();
        while (lo < hi && image[lo] == before[lo])
            ++lo;
        while (hi > lo && image[hi - 1] == before[hi - 1])
            --hi;
        if (hi > lo) {
            auto w = detail::disk_write(_disk, base + lo, image.data() + lo, hi - lo);
            if (!w)
                return unexpected(w.error());
        }
        if (counts)
            std::memcpy(counts, c3, sizeof c3);
        return {};
    }

protected:
    EngineBlockDevice(IDisk& disk, std::shared_ptr<Logger> logger, uint32_t type, uint32_t bs, uint32_t t,
        uint64_t poly, int device, const char* log_name)
        : _disk(disk)
        , _logger(std::move(logger))
        , _type(type)
        , _eng(type, bs, t, poly, device)
        , _raw(_eng.raw())
        , _ds(_eng.data())
        , _log_name(log_name)
    {
    }

    bool has_spill() const { return _type == PPFS_ECC_REED_SOLOMON && _raw > 0 && _raw < 255; }
    size_t spill_stride() const { return 256 - std::min<size_t>(_raw, 255); }

    void log(block_index_t b)
    {
        if (_logger && _log_name)
            _logger->logEvent(ErrorCorrectionEvent(_log_name, b));
    }

    // The reference's write-back of a corrected block (old = raw as read, fixed = corrected).
    expected<void> write_back(block_index_t b, const uint8_t* old, const uint8_t* fixed, const uint8_t* spill)
    {
        if (_type == PPFS_ECC_REED_SOLOMON) {
            // rs_block_device.cpp:171-180: log, then write the whole corrected codeword (and,
            // for shortened codes, what its polynomial holds past n); the result is ignored
            log(b);
            std::vector<uint8_t> wbuf(fixed, fixed + _raw);
            if (spill && spill[0])
                wbuf.insert(wbuf.end(), spill + 1, spill + 1 + spill[0]);
            (void)detail::disk_write(_disk, (size_t)b * _raw, wbuf.data(), wbuf.size());
            return {};
        }
        // hamming_block_device.cpp:41-57: write back only the flipped byte, then log
        size_t byte = 0;
        while (byte < _raw && old[byte] == fixed[byte])
            ++byte;
        if (byte == _raw)
            byte = 0;
        auto w = detail::disk_write(_disk, (size_t)b * _raw + byte, fixed + byte, 1);
        if (!w)
            return unexpected(w.error());
        log(b);
        return {};
    }

    // _fixBlockAndExtract / _readAndCheckRaw / _readAndFixBlock for one block; raw is replaced
    // by the (fixed) old block, dec receives the payload.
    expected<void> check_fix(block_index_t b, uint8_t* raw, uint8_t* dec)
    {
        std::vector<uint8_t> fixed(raw, raw + _raw), spill;
        uint8_t status = 0;
        if (has_spill())
            spill.assign(spill_stride(), 0);
        const int wb = (_type == PPFS_ECC_REED_SOLOMON || _type == PPFS_ECC_HAMMING) ? 1 : 0;
        if (!EccEngine::ok(ppfs_ecc_decode_host(_eng.ctx(), fixed.data(), dec, &status, 1, wb,
                               spill.empty() ? nullptr : spill.data()),
                "decode"))
            return unexpected(FsError::Disk_IOError);
        if (status == PPFS_ECC_CORRECTION_ERROR)
            return unexpected(FsError::BlockDevice_CorrectionError);
        if (status == PPFS_ECC_CORRECTED && wb) {
            auto w = write_back(b, raw, fixed.data(), spill.empty() ? nullptr : spill.data());
            if (!w)
                return w;
        }
        std::memcpy(raw, fixed.data(), _raw);
        return {};
    }

    IDisk& _disk;
    std::shared_ptr<Logger> _logger;
    uint32_t _type;
    EccEngine _eng;
    size_t _raw, _ds;
    const char* _log_name;
};

class ReedSolomonBlockDevice : public EngineBlockDevice {
public:
    // raw_block_size is clamped to 255 and correctable_bytes to raw/2 (rs_block_device.cpp:52-60)
    ReedSolomonBlockDevice(IDisk& disk, size_t raw_block_size, size_t correctable_bytes,
        std::shared_ptr<Logger> logger = nullptr, int device = 0)
        : EngineBlockDevice(disk, std::move(logger), PPFS_ECC_REED_SOLOMON, (uint32_t)raw_block_size,
            (uint32_t)correctable_bytes, 0, device, "ReedSolomon")
    {
    }
};

class CrcBlockDevice : public EngineBlockDevice {
public:
    CrcBlockDevice(CrcPolynomial polynomial, IDisk& disk, size_t block_size, std::shared_ptr<Logger> logger = nullptr,
        int device = 0)
        : EngineBlockDevice(disk, std::move(logger), PPFS_ECC_CRC, (uint32_t)block_size, 0,
            polynomial.getExplicitPolynomial(), device, nullptr)
    {
    }
};

class HammingBlockDevice : public EngineBlockDevice {
public:
    HammingBlockDevice(int block_size_power, IDisk& disk, std::shared_ptr<Logger> logger = nullptr, int device = 0)
        : EngineBlockDevice(disk, std::move(logger), PPFS_ECC_HAMMING, 1u << block_size_power, 0, 0, device,
            "Hamming")
    {
    }
};

class ParityBlockDevice : public EngineBlockDevice {
public:
    ParityBlockDevice(int block_size, IDisk& disk, std::shared_ptr<Logger> logger = nullptr, int device = 0)
        : EngineBlockDevice(disk, std::move(logger), PPFS_ECC_PARITY, (uint32_t)block_size, 0, 0, device, nullptr)
    {
    }
};

} // namespace ppfs_gpu
