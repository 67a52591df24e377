// test_block_devices.cpp -- the C++ host adapter (include/ppfs_gpu/block_device.hpp) on the GPU.
//
// Part 1 restates the reference's own block-device unit tests with the same names and checks:
//   unit_tests/test_rs_block_device.cpp, test_crc_block_device.cpp (device tests),
//   test_hamming_block_device.cpp, test_parity_block_device.cpp, test_stack_disk.cpp.
// Part 2 is differential: random sequences of formatBlock / writeBlock (any offset and length)
// / readBlock / readBlocks / writeBlocks / scrub / raw corruption applied to the adapter and to the
// oracle's device model (oracle/ppfs_oracle.c oracle_dev_*, the reference's per-block
// semantics restated in C; TEST INFRASTRUCTURE ONLY), comparing every return value, every
// payload, the correction log and the whole disk image after each operation.
//
// Exit status 0 and "ALL PASSED" on success.  Needs a GPU (the adapter has no CPU fallback).
#include "ppfs_gpu/block_device.hpp"

#include <array>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

using namespace ppfs_gpu;

// ---- minimal test harness ------------------------------------------------------------------
static int g_fail = 0, g_checks = 0;
static const char* g_test = "";
#define EXPECT_TRUE(c)                                                                                   \
    do {                                                                                                 \
        ++g_checks;                                                                                      \
        if (!(c)) {                                                                                      \
            ++g_fail;                                                                                    \
            std::fprintf(stderr, "FAIL %s:%d [%s]: %s\n", __FILE__, __LINE__, g_test, #c);               \
        }                                                                                                \
    } while (0)
#define ASSERT_TRUE(c)                                                                                   \
    do {                                                                                                 \
        ++g_checks;                                                                                      \
        if (!(c)) {                                                                                      \
            ++g_fail;                                                                                    \
            std::fprintf(stderr, "FAIL %s:%d [%s]: %s (fatal)\n", __FILE__, __LINE__, g_test, #c);       \
            return;                                                                                      \
        }                                                                                                \
    } while (0)
#define EXPECT_FALSE(c) EXPECT_TRUE(!(c))
#define ASSERT_FALSE(c) ASSERT_TRUE(!(c))
#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))
#define ASSERT_EQ(a, b) ASSERT_TRUE((a) == (b))

struct TestCase {
    const char* name;
    std::function<void()> fn;
};
static std::vector<TestCase>& registry()
{
    static std::vector<TestCase> r;
    return r;
}
struct Reg {
    Reg(const char* n, std::function<void()> f) { registry().push_back({ n, std::move(f) }); }
};
#define TEST(suite, name)                                                                                \
    static void suite##_##name();                                                                        \
    static Reg reg_##suite##_##name(#suite "." #name, suite##_##name);                                   \
    static void suite##_##name()

// ---- oracle device model (test infrastructure) ---------------------------------------------
extern "C" {
void* oracle_dev_create(int type, int block_size, int t, uint64_t explicit_poly, uint8_t* disk, size_t disk_size,
    int32_t* log, size_t log_cap);
void oracle_dev_destroy(void* h);
size_t oracle_dev_log_len(void* h);
int oracle_dev_format(void* h, unsigned block);
int oracle_dev_read(void* h, int block, size_t offset, size_t nbytes, size_t out_capacity, uint8_t* out,
    size_t* out_len);
int oracle_dev_write(void* h, int block, size_t offset, const uint8_t* data, size_t len, size_t* written);
}

// =============================================================================================
// Part 1: the reference's unit tests
// =============================================================================================
static void flipBit(StackDisk<>& disk, size_t bitIndex)
{
    std::array<uint8_t, 1> b;
    static_vector<uint8_t> bytes(b.data(), 1);
    auto r = disk.read(bitIndex / 8, 1, bytes);
    if (!r.has_value())
        std::abort();
    bytes[0] ^= static_cast<std::uint8_t>(1 << (bitIndex % 8));
    if (!disk.write(bitIndex / 8, bytes).has_value())
        std::abort();
}
static std::mt19937 g_gen(12345);
static size_t randomBit(size_t maxBits) { return std::uniform_int_distribution<size_t>(0, maxBits - 1)(g_gen); }

template <class Dev> static void rs_corrupt_and_read(StackDisk<>& disk, Dev& rs, std::vector<std::pair<int, uint8_t>> bad)
{
    auto data_size = rs.dataSize();
    std::array<uint8_t, 512> data_buffer;
    std::fill(data_buffer.begin(), data_buffer.begin() + data_size, static_cast<std::uint8_t>(0xAB));
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), data_size);
    ASSERT_TRUE(rs.formatBlock(0).has_value());
    ASSERT_TRUE(rs.writeBlock(data, DataLocation(0, 0)).has_value());
    std::array<uint8_t, 512> raw_buffer;
    static_vector<uint8_t> raw(raw_buffer.data(), raw_buffer.size());
    raw.resize(rs.rawBlockSize());
    ASSERT_TRUE(disk.read(0, rs.rawBlockSize(), raw).has_value());
    for (auto& p : bad)
        raw[p.first] = p.second;
    ASSERT_TRUE(disk.write(0, raw).has_value());
    std::array<uint8_t, 512> read_buffer;
    static_vector<uint8_t> fixed(read_buffer.data(), read_buffer.size());
    ASSERT_TRUE(rs.readBlock({ 0, 0 }, data_size, fixed).has_value());
    for (size_t i = 0; i < data_size; i++)
        EXPECT_EQ(fixed[i], data[i]);
}

TEST(ReedSolomonBlockDevice, BasicReadWrite)
{
    StackDisk<> disk;
    ReedSolomonBlockDevice rs(disk, 255, 2);
    rs_corrupt_and_read(disk, rs, {});
}
TEST(ReedSolomonBlockDevice, SingleByteError)
{
    StackDisk<> disk;
    ReedSolomonBlockDevice rs(disk, 255, 1);
    rs_corrupt_and_read(disk, rs, { { 120, 0x00 } });
}
TEST(ReedSolomonBlockDevice, DoubleByteError)
{
    StackDisk<> disk;
    ReedSolomonBlockDevice rs(disk, 255, 2);
    rs_corrupt_and_read(disk, rs, { { 10, 0xEE }, { 200, 0x44 } });
}
TEST(ReedSolomonBlockDevice, TripleByteError)
{
    StackDisk<> disk;
    ReedSolomonBlockDevice rs(disk, 255, 3);
    rs_corrupt_and_read(disk, rs, { { 10, 0xEE }, { 100, 0x61 }, { 200, 0x44 } });
}

TEST(CrcBlockDevice, Compiles)
{
    StackDisk<> disk;
    CrcBlockDevice crc(CrcPolynomial::MsgImplicit(0xea), disk, 256);
    EXPECT_TRUE(crc.dataSize() > 0);
}
TEST(CrcBlockDevice, ReadsAndWrites)
{
    StackDisk<> disk;
    auto poly = CrcPolynomial::MsgImplicit(0xea);
    CrcBlockDevice crc(poly, disk, 256);
    auto data_size = crc.dataSize();
    std::array<uint8_t, 512> data_buffer;
    std::fill(data_buffer.begin(), data_buffer.begin() + data_size, static_cast<std::uint8_t>(0x55));
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), data_size);
    ASSERT_TRUE(crc.formatBlock(0).has_value());
    ASSERT_TRUE(crc.writeBlock(data, DataLocation(0, 0)).has_value());
    std::array<uint8_t, 512> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    ASSERT_TRUE(crc.readBlock({ 0, 0 }, data_size, read_data).has_value());
    for (size_t i = 0; i < data_size; i++)
        EXPECT_EQ(data[i], read_data[i]);
}
static void crc_flip_test(uint64_t implicit_poly, size_t bs, std::vector<std::pair<size_t, uint8_t>> writes)
{
    StackDisk<> disk;
    CrcBlockDevice crc(CrcPolynomial::MsgImplicit(implicit_poly), disk, bs);
    auto data_size = crc.dataSize();
    std::array<uint8_t, 1024> data_buffer;
    std::fill(data_buffer.begin(), data_buffer.begin() + data_size, static_cast<std::uint8_t>(0x00));
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), data_size);
    ASSERT_TRUE(crc.formatBlock(0).has_value());
    ASSERT_TRUE(crc.writeBlock(data, DataLocation(0, 0)).has_value());
    for (auto& w : writes) {
        std::array<uint8_t, 1> b = { w.second };
        static_vector<uint8_t> v(b.data(), 1, 1);
        ASSERT_TRUE(disk.write(w.first, v).has_value());
    }
    std::array<uint8_t, 1024> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    auto read_ret = crc.readBlock({ 0, 0 }, data_size, read_data);
    EXPECT_FALSE(read_ret.has_value());
    EXPECT_TRUE(read_ret.error() == FsError::BlockDevice_CorrectionError);
}
TEST(CrcBlockDevice, FindsError) { crc_flip_test(0xea, 256, { { 1, 0x01 } }); }
TEST(CrcBlockDevice, FindEnoughErrors) { crc_flip_test(0xc1acf, 512, { { 1, 0x01 }, { 111, 0x08 }, { 200, 0x02 } }); }
TEST(CrcBlockDevice, FindEvenMoreErrors)
{
    crc_flip_test(0x9960034c, 512, { { 1, 0x01 }, { 111, 0x08 }, { 200, 0x02 }, { 11, 0x08 }, { 20, 0x02 } });
}

TEST(HammingBlockDevice, BasicWriteRead)
{
    StackDisk<> disk;
    HammingBlockDevice hbd(4, disk);
    std::array<uint8_t, 16> data_buffer = { 'h', 'e', 'l', 'l', 'o' };
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), 5);
    auto w = hbd.writeBlock(data, DataLocation(0, 0));
    ASSERT_TRUE(w.has_value());
    EXPECT_EQ(w.value(), (size_t)5);
    std::array<uint8_t, 16> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    ASSERT_TRUE(hbd.readBlock(DataLocation(0, 0), 5, read_data).has_value());
    ASSERT_EQ(read_data.size(), (size_t)5);
    for (size_t i = 0; i < 5; ++i)
        EXPECT_EQ(read_data[i], data[i]);
}
TEST(HammingBlockDevice, SingleBitErrorIsCorrected)
{
    StackDisk<> disk;
    HammingBlockDevice hbd(4, disk);
    DataLocation loc(0, 0);
    std::array<uint8_t, 16> data_buffer = { 's', 'l', 'a', 'y' };
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), 4);
    ASSERT_TRUE(hbd.writeBlock(data, loc).has_value());
    flipBit(disk, randomBit(hbd.dataSize() * 8));
    std::array<uint8_t, 16> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    ASSERT_TRUE(hbd.readBlock(loc, data.size(), read_data).has_value());
    for (size_t i = 0; i < data.size(); ++i)
        EXPECT_EQ(read_data[i], data[i]);
}
TEST(HammingBlockDevice, DoubleBitErrorTriggersFailure)
{
    StackDisk<> disk;
    HammingBlockDevice hbd(4, disk);
    DataLocation loc(0, 0);
    std::array<uint8_t, 16> data_buffer = { 's', 'l', 'a', 'y' };
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), 4);
    ASSERT_TRUE(hbd.writeBlock(data, loc).has_value());
    size_t totalBits = hbd.dataSize() * 8;
    size_t bit1 = randomBit(totalBits), bit2 = randomBit(totalBits);
    while (bit2 == bit1)
        bit2 = randomBit(totalBits);
    flipBit(disk, bit1);
    flipBit(disk, bit2);
    std::array<uint8_t, 16> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    auto read_res = hbd.readBlock(loc, data.size(), read_data);
    ASSERT_FALSE(read_res.has_value());
    EXPECT_TRUE(read_res.error() == FsError::BlockDevice_CorrectionError);
}
TEST(HammingBlockDevice, MultipleRandomSingleBitCorrections)
{
    for (int i = 0; i < 10; ++i) {
        StackDisk<> disk;
        HammingBlockDevice hbd(4, disk);
        DataLocation loc(0, 0);
        std::string msg = "Round" + std::to_string(i);
        std::array<uint8_t, 16> data_buffer;
        for (size_t j = 0; j < msg.size(); j++)
            data_buffer[j] = static_cast<std::uint8_t>(msg[j]);
        static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), msg.size());
        ASSERT_TRUE(hbd.writeBlock(data, loc).has_value());
        flipBit(disk, randomBit(hbd.dataSize() * 8));
        std::array<uint8_t, 16> read_buffer;
        static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
        ASSERT_TRUE(hbd.readBlock(loc, data.size(), read_data).has_value());
        std::string decoded(reinterpret_cast<const char*>(read_data.data()), read_data.size());
        ASSERT_TRUE(decoded == msg);
    }
}

TEST(ParityBlockDevice, BasicReadWrite)
{
    StackDisk<> disk;
    ParityBlockDevice parity(256, disk);
    auto data_size = parity.dataSize();
    std::array<uint8_t, 512> data_buffer;
    std::fill(data_buffer.begin(), data_buffer.begin() + data_size, static_cast<std::uint8_t>(0xAA));
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), data_size);
    ASSERT_TRUE(parity.formatBlock(0).has_value());
    ASSERT_TRUE(parity.writeBlock(data, DataLocation(0, 0)).has_value());
    std::array<uint8_t, 512> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    ASSERT_TRUE(parity.readBlock({ 0, 0 }, data_size, read_data).has_value());
    ASSERT_EQ(read_data.size(), data_size);
    for (size_t i = 0; i < data_size; i++)
        EXPECT_EQ(data[i], read_data[i]);
}
TEST(ParityBlockDevice, DetectsSingleBitFlip)
{
    StackDisk<> disk;
    ParityBlockDevice parity(256, disk);
    auto data_size = parity.dataSize();
    std::array<uint8_t, 512> data_buffer;
    std::fill(data_buffer.begin(), data_buffer.begin() + data_size, static_cast<std::uint8_t>(0x55));
    static_vector<uint8_t> data(data_buffer.data(), data_buffer.size(), data_size);
    ASSERT_TRUE(parity.formatBlock(0).has_value());
    ASSERT_TRUE(parity.writeBlock(data, DataLocation(0, 0)).has_value());
    std::array<uint8_t, 512> raw_buffer;
    static_vector<uint8_t> raw(raw_buffer.data(), raw_buffer.size());
    raw.resize(parity.rawBlockSize());
    ASSERT_TRUE(disk.read(0, parity.rawBlockSize(), raw).has_value());
    raw[10] ^= static_cast<std::uint8_t>(4);
    ASSERT_TRUE(disk.write(0, raw).has_value());
    std::array<uint8_t, 512> read_buffer;
    static_vector<uint8_t> read_data(read_buffer.data(), read_buffer.size());
    EXPECT_FALSE(parity.readBlock({ 0, 0 }, data_size, read_data).has_value());
}

TEST(StackDisk, OutOfBounds)
{
    StackDisk<> d;
    std::array<uint8_t, 3> b;
    static_vector<uint8_t> v(b.data(), 3, 3);
    EXPECT_FALSE(d.write(d.size() - 2, v).has_value());
    EXPECT_FALSE(d.read(d.size() - 2, 3, v).has_value());
    EXPECT_TRUE(d.read(d.size() - 3, 3, v).has_value());
}

// =============================================================================================
// Part 2: differential sequences against the oracle's device model
// =============================================================================================
struct Cfg {
    const char* name;
    int type;
    int bs;
    int t;
    uint64_t poly; // explicit
};

static std::unique_ptr<IBlockDevice> make_dev(const Cfg& c, IDisk& disk, std::shared_ptr<Logger> lg)
{
    switch (c.type) {
    case PPFS_ECC_REED_SOLOMON:
        return std::make_unique<ReedSolomonBlockDevice>(disk, c.bs, c.t, lg);
    case PPFS_ECC_CRC:
        return std::make_unique<CrcBlockDevice>(CrcPolynomial::MsgExplicit(c.poly), disk, c.bs, lg);
    case PPFS_ECC_HAMMING: {
        int p = 0;
        while ((1 << (p + 1)) <= c.bs)
            ++p;
        return std::make_unique<HammingBlockDevice>(p, disk, lg);
    }
    case PPFS_ECC_PARITY:
        return std::make_unique<ParityBlockDevice>(c.bs, disk, lg);
    default:
        return std::make_unique<RawBlockDevice>(c.bs, disk);
    }
}

// Disks for the differential runs: the in-memory disk with the engine batch calls in place on its
// image (mapped) or through a copy (not mapped), and the mmap'd file disk.
template <bool MAP> struct TestStackDisk : public StackDisk<20> {
    uint8_t* mapped() override { return MAP ? image() : nullptr; }
};
struct TestFileDisk : public MappedFileDisk {
    TestFileDisk()
    {
        char path[] = "/tmp/ppfs_mfd_XXXXXX";
        const int fd = mkstemp(path);
        if (fd >= 0)
            ::close(fd);
        EXPECT_TRUE(create(path, size_t(1) << 20).has_value());
        EXPECT_TRUE(!create(path, 16).has_value()); // file_disk.cpp:37-38: already open
        ::unlink(path);                             // the mapping stays valid
    }
    uint8_t* image() { return mapped(); }
};

template <class D> static void differential(const Cfg& c, uint64_t seed, int nops)
{
    constexpr size_t NB = 48;
    D disk; // 1 MiB
    auto lg = std::make_shared<Logger>();
    auto dev = make_dev(c, disk, lg);
    const size_t raw = dev->rawBlockSize(), ds = dev->dataSize();
    const size_t span = NB * raw;
    std::vector<uint8_t> odisk(disk.size(), 0);
    std::vector<int32_t> olog(1 << 16);
    void* od = oracle_dev_create(c.type, c.bs, c.t, c.poly, odisk.data(), odisk.size(), olog.data(), olog.size());
    std::mt19937_64 rng(seed);
    auto rnd = [&](uint64_t n) { // n = 0 (no payload: Hamming power 0, 1-byte parity) gives 0
        const uint64_t v = rng();
        return n ? v % n : (uint64_t)0;
    };
    auto same_disk = [&]() { return std::memcmp(disk.image(), odisk.data(), odisk.size()) == 0; };
    auto same_log = [&]() {
        if (lg->events.size() != oracle_dev_log_len(od))
            return false;
        for (size_t i = 0; i < lg->events.size(); ++i)
            if ((int32_t)lg->events[i].block_index != olog[i])
                return false;
        return true;
    };
    // start from formatted blocks with random payloads written (valid codewords)
    for (size_t b = 0; b < NB; ++b) {
        EXPECT_TRUE(dev->formatBlock((unsigned)b).has_value());
        oracle_dev_format(od, (unsigned)b);
    }
    std::vector<uint8_t> buf(NB * 4096), obuf(NB * 4096);
    for (int op = 0; op < nops; ++op) {
        const int kind = (int)rnd(9);
        const int b = (int)rnd(NB + 1); // NB: past the used range (still on the disk)
        if (kind == 0) { // formatBlock
            auto r = dev->formatBlock((unsigned)b);
            int orr = oracle_dev_format(od, (unsigned)b);
            EXPECT_EQ(r.has_value(), orr == 0);
        } else if (kind <= 2) { // writeBlock, any offset / length
            const size_t off = rnd(4) == 0 ? rnd(ds) : 0;
            const size_t len = rnd(3) == 0 ? rnd(ds + 8) : ds;
            for (size_t i = 0; i < len; ++i)
                buf[i] = (uint8_t)rng();
            static_vector<uint8_t> v(buf.data(), len, len);
            auto r = dev->writeBlock(v, DataLocation(b, off));
            size_t ow = 0;
            int orr = oracle_dev_write(od, b, off, buf.data(), len, &ow);
            EXPECT_EQ(r.has_value(), orr == 0);
            if (r.has_value() && orr == 0)
                EXPECT_EQ(r.value(), ow);
            if (!r.has_value() && orr != 0)
                EXPECT_EQ((int)r.error(), orr);
        } else if (kind <= 4) { // readBlock with random capacity / size
            const size_t off = rnd(4) == 0 ? rnd(ds) : 0;
            const size_t n = rnd(3) == 0 ? rnd(ds + 8) : ds;
            const size_t cap = rnd(8) == 0 ? (n ? n - 1 : 0) : 4096;
            static_vector<uint8_t> v(buf.data(), cap);
            auto r = dev->readBlock(DataLocation(b, off), n, v);
            size_t olen = 0;
            int orr = oracle_dev_read(od, b, off, n, cap, obuf.data(), &olen);
            EXPECT_EQ(r.has_value(), orr == 0);
            if (r.has_value() && orr == 0) {
                EXPECT_EQ(v.size(), olen);
                EXPECT_TRUE(std::memcmp(buf.data(), obuf.data(), olen) == 0);
            }
            if (!r.has_value() && orr != 0)
                EXPECT_EQ((int)r.error(), orr);
        } else if (kind == 5) { // corrupt: random bit flips / byte overwrites in a few blocks
            const int nblk = 1 + (int)rnd(4);
            for (int k = 0; k < nblk; ++k) {
                const size_t blk = rnd(NB);
                const int nerr = (int)rnd(c.type == PPFS_ECC_REED_SOLOMON ? c.t + 3 : 3);
                for (int e = 0; e < nerr; ++e) {
                    const size_t pos = blk * raw + rnd(raw);
                    const uint8_t m = c.type == PPFS_ECC_REED_SOLOMON ? (uint8_t)(1 + rnd(255)) : (uint8_t)(1u << rnd(8));
                    disk.image()[pos] ^= m;
                    odisk[pos] ^= m;
                }
            }
        } else if (kind == 6) { // readBlocks == per-block readBlock loop
            const size_t first = rnd(NB), cnt = 1 + rnd(NB - first);
            std::vector<uint8_t> err(cnt);
            auto r = dev->readBlocks((block_index_t)first, cnt, buf.data(), err.data());
            EXPECT_TRUE(r.has_value());
            for (size_t i = 0; i < cnt; ++i) {
                size_t olen = 0;
                int orr = oracle_dev_read(od, (int)(first + i), 0, ds, 4096, obuf.data(), &olen);
                EXPECT_EQ((int)err[i], orr);
                if (orr == 0)
                    EXPECT_TRUE(std::memcmp(buf.data() + i * ds, obuf.data(), ds) == 0);
            }
        } else if (kind == 8) { // scrub == per-block readBlock loop, payloads dropped
            const size_t first = rnd(NB), cnt = 1 + rnd(NB - first);
            std::vector<uint8_t> err(cnt);
            size_t counts[3] = { 0, 0, 0 };
            auto r = dev->scrub((block_index_t)first, cnt, counts, err.data());
            EXPECT_TRUE(r.has_value());
            size_t failed = 0;
            for (size_t i = 0; i < cnt; ++i) {
                size_t olen = 0;
                int orr = oracle_dev_read(od, (int)(first + i), 0, ds, 4096, obuf.data(), &olen);
                EXPECT_EQ((int)err[i], orr);
                failed += orr != 0;
            }
            EXPECT_EQ(counts[0] + counts[1] + counts[2], cnt);
            EXPECT_EQ(counts[2], failed);
        } else { // writeBlocks == per-block writeBlock loop
            const size_t first = rnd(NB), cnt = 1 + rnd(NB - first);
            for (size_t i = 0; i < cnt * ds; ++i)
                buf[i] = (uint8_t)rng();
            std::vector<uint8_t> err(cnt);
            auto r = dev->writeBlocks((block_index_t)first, cnt, buf.data(), err.data());
            EXPECT_TRUE(r.has_value());
            for (size_t i = 0; i < cnt; ++i) {
                size_t ow = 0;
                int orr = oracle_dev_write(od, (int)(first + i), 0, buf.data() + i * ds, ds, &ow);
                EXPECT_EQ((int)err[i], orr);
            }
        }
        if (!same_disk() || !same_log()) {
            ++g_fail;
            std::fprintf(stderr, "FAIL [%s] %s seed %llu: state diverged after op %d (kind %d, block %d)\n", g_test,
                c.name, (unsigned long long)seed, op, kind, b);
            break;
        }
        ++g_checks;
    }
    (void)span;
    oracle_dev_destroy(od);
}

static const Cfg kCfgs[] = {
    { "rs255_t1", PPFS_ECC_REED_SOLOMON, 255, 1, 0 },
    { "rs512_t3", PPFS_ECC_REED_SOLOMON, 512, 3, 0 },
    { "rs256_t4", PPFS_ECC_REED_SOLOMON, 256, 4, 0 },
    { "rs4096_t16", PPFS_ECC_REED_SOLOMON, 4096, 16, 0 },
    { "rs64_t3_shortened", PPFS_ECC_REED_SOLOMON, 64, 3, 0 },
    { "rs128_t10_shortened", PPFS_ECC_REED_SOLOMON, 128, 10, 0 },
    { "crc512_0x9960034c", PPFS_ECC_CRC, 512, 0, (0x9960034cull << 1) + 1 },
    { "crc256_0xea", PPFS_ECC_CRC, 256, 0, (0xeaull << 1) + 1 },
    { "crc512_0xc1acf", PPFS_ECC_CRC, 512, 0, (0xc1acfull << 1) + 1 },
    { "crc100_deg3", PPFS_ECC_CRC, 100, 0, 0xb },
    { "crc4096_deg32", PPFS_ECC_CRC, 4096, 0, (0x9960034cull << 1) + 1 },
    { "hamming1_pow0", PPFS_ECC_HAMMING, 1, 0, 0 },
    { "hamming2_pow1", PPFS_ECC_HAMMING, 2, 0, 0 },
    { "hamming4_pow2", PPFS_ECC_HAMMING, 4, 0, 0 },
    { "hamming8", PPFS_ECC_HAMMING, 8, 0, 0 },
    { "hamming16", PPFS_ECC_HAMMING, 16, 0, 0 },
    { "hamming512", PPFS_ECC_HAMMING, 512, 0, 0 },
    { "hamming4096", PPFS_ECC_HAMMING, 4096, 0, 0 },
    { "parity1", PPFS_ECC_PARITY, 1, 0, 0 },
    { "parity256", PPFS_ECC_PARITY, 256, 0, 0 },
    { "parity4096", PPFS_ECC_PARITY, 4096, 0, 0 },
    { "raw512", PPFS_ECC_NONE, 512, 0, 0 },
};

TEST(Differential, AllCodecsVsOracleDeviceModel)
{
    for (const Cfg& c : kCfgs)
        for (uint64_t seed = 1; seed <= 3; ++seed)
            differential<TestStackDisk<true>>(c, seed * 7919 + (uint64_t)c.type, 160);
}

TEST(Differential, AllCodecsThroughCopiesVsOracleDeviceModel)
{
    for (const Cfg& c : kCfgs)
        for (uint64_t seed = 1; seed <= 2; ++seed)
            differential<TestStackDisk<false>>(c, seed * 104729 + (uint64_t)c.type, 160);
}

TEST(Differential, MappedFileDiskVsOracleDeviceModel)
{
    for (const Cfg& c : kCfgs)
        differential<TestFileDisk>(c, 31337 + (uint64_t)c.type, 160);
}

// readBlocks over a range that runs past the disk end == readBlock of every block: the in-range
// blocks are decoded (and written back / logged), the off-disk ones report Disk_OutOfBounds
template <class D> static void straddle(const Cfg& c)
{
    D disk;
    auto lg = std::make_shared<Logger>();
    auto dev = make_dev(c, disk, lg);
    const size_t raw = dev->rawBlockSize(), ds = dev->dataSize(), nb = dev->numOfBlocks();
    std::vector<uint8_t> odisk(disk.size(), 0);
    std::vector<int32_t> olog(1 << 12);
    void* od = oracle_dev_create(c.type, c.bs, c.t, c.poly, odisk.data(), odisk.size(), olog.data(), olog.size());
    std::mt19937_64 rng(77 + (uint64_t)c.type);
    const size_t first = nb - 5, cnt = 9; // 5 blocks on the disk, 4 past its end
    std::vector<uint8_t> pl(ds);
    for (size_t b = first; b < nb; ++b) {
        for (auto& x : pl)
            x = (uint8_t)rng();
        static_vector<uint8_t> v(pl.data(), ds, ds);
        EXPECT_TRUE(dev->writeBlock(v, DataLocation((int)b, 0)).has_value());
        size_t ow = 0;
        oracle_dev_write(od, (int)b, 0, pl.data(), ds, &ow);
    }
    for (size_t b = first; b < nb; b += 2) { // one error in every other block
        const size_t pos = b * raw + (size_t)(rng() % raw);
        const uint8_t m = c.type == PPFS_ECC_REED_SOLOMON ? (uint8_t)(1 + rng() % 255) : (uint8_t)(1u << (rng() % 8));
        disk.image()[pos] ^= m;
        odisk[pos] ^= m;
    }
    std::vector<uint8_t> out(cnt * ds, 0xEE), err(cnt, 0xEE), obuf(4096);
    EXPECT_TRUE(dev->readBlocks((block_index_t)first, cnt, out.data(), err.data()).has_value());
    for (size_t i = 0; i < cnt; ++i) {
        size_t olen = 0;
        const int orr = oracle_dev_read(od, (int)(first + i), 0, ds, 4096, obuf.data(), &olen);
        EXPECT_EQ((int)err[i], orr);
        if (orr == 0)
            EXPECT_TRUE(std::memcmp(out.data() + i * ds, obuf.data(), ds) == 0);
    }
    EXPECT_TRUE(std::memcmp(disk.image(), odisk.data(), odisk.size()) == 0);
    EXPECT_EQ(lg->events.size(), oracle_dev_log_len(od));
    oracle_dev_destroy(od);
    ++g_checks;
}

TEST(Differential, ReadBlocksStraddlingDiskEnd)
{
    for (const Cfg& c : kCfgs) {
        if (c.type == PPFS_ECC_NONE)
            continue;
        straddle<TestStackDisk<true>>(c);
        straddle<TestStackDisk<false>>(c);
    }
}

// An engine error reaches the caller as FsError::Disk_IOError (no throw, no abort): here the
// engine cannot be created at all (no such device), so every call of the device fails that way.
TEST(EngineErrors, PropagateAsDiskIOError)
{
    TestStackDisk<true> disk;
    ReedSolomonBlockDevice rs(disk, 512, 3, nullptr, /*device=*/4096);
    EXPECT_EQ(rs.numOfBlocks(), (size_t)0);
    uint8_t buf[512] = { 0 };
    static_vector<uint8_t> v(buf, sizeof buf, 16);
    auto w = rs.writeBlock(v, DataLocation(0, 0));
    EXPECT_TRUE(!w.has_value() && w.error() == FsError::Disk_IOError);
    static_vector<uint8_t> r(buf, sizeof buf);
    auto rr = rs.readBlock(DataLocation(0, 0), 16, r);
    EXPECT_TRUE(!rr.has_value() && rr.error() == FsError::Disk_IOError);
    uint8_t err[2] = { 0, 0 };
    auto rb = rs.readBlocks(0, 2, buf, err);
    EXPECT_TRUE(!rb.has_value() && rb.error() == FsError::Disk_IOError);
    auto wb = rs.writeBlocks(0, 1, buf, err);
    EXPECT_TRUE(!wb.has_value() && wb.error() == FsError::Disk_IOError);
    size_t counts[3];
    auto sc = rs.scrub(0, 1, counts, err);
    EXPECT_TRUE(!sc.has_value());
    CrcBlockDevice crc(CrcPolynomial::MsgImplicit(0x9960034c), disk, 512, nullptr, 4096);
    auto f = crc.formatBlock(0);
    EXPECT_TRUE(!f.has_value() && f.error() == FsError::Disk_IOError);
}

TEST(MappedFileDisk, FileDiskChecks)
{
    MappedFileDisk d;
    uint8_t buf[64];
    static_vector<uint8_t> v(buf, 64);
    EXPECT_EQ((int)d.read(0, 8, v).error(), (int)FsError::Disk_IOError); // not open
    EXPECT_EQ((int)d.open("/nonexistent/ppfs").error(), (int)FsError::Disk_IOError);
    char path[] = "/tmp/ppfs_mfd_XXXXXX";
    const int fd = mkstemp(path);
    EXPECT_TRUE(fd >= 0);
    ::close(fd);
    EXPECT_TRUE(d.create(path, 4096).has_value());
    EXPECT_EQ(d.size(), (size_t)4096);
    EXPECT_EQ((int)d.read(4090, 8, v).error(), (int)FsError::Disk_OutOfBounds);
    static_vector<uint8_t> small(buf, 4);
    EXPECT_EQ((int)d.read(0, 8, small).error(), (int)FsError::Disk_InvalidRequest);
    for (int i = 0; i < 64; ++i)
        buf[i] = (uint8_t)(i * 7);
    static_vector<uint8_t> w(buf, 64, 64);
    EXPECT_EQ(d.write(100, w).value(), (size_t)64);
    EXPECT_EQ((int)d.write(4090, w).error(), (int)FsError::Disk_OutOfBounds);
    d.close();
    MappedFileDisk e; // reopen: the bytes reached the file
    EXPECT_TRUE(e.open(path).has_value());
    uint8_t rb[64] = { 0 };
    static_vector<uint8_t> r(rb, 64);
    EXPECT_TRUE(e.read(100, 64, r).has_value());
    EXPECT_TRUE(std::memcmp(rb, buf, 64) == 0);
    e.close();
    ::unlink(path);
}

int main(int argc, char** argv)
{
    const char* only = argc > 1 ? argv[1] : nullptr;
    for (auto& tc : registry()) {
        if (only && std::string(tc.name).find(only) == std::string::npos)
            continue;
        g_test = tc.name;
        const int before = g_fail;
        tc.fn();
        std::printf("%s %s\n", g_fail == before ? "ok  " : "FAIL", tc.name);
    }
    std::printf("%d checks, %d failures\n", g_checks, g_fail);
    if (g_fail == 0)
        std::printf("ALL PASSED\n");
    return g_fail == 0 ? 0 : 1;
}
