// bench_blockdevice.cpp -- the reference's performance_tests/bench_blockdevice.cpp workload on the
// GPU-backed adapter (include/ppfs_gpu/block_device.hpp), plus the batched form.
//
// Reference cases (same devices and parameters): block_size 256 -- raw, CRC MsgImplicit(0xea),
// Hamming 2^8, RS t=16 -- readBlock({0,0}, n) and writeBlock(n bytes, {1,0}) for n = 1,2,4..256.
// Reported like google/benchmark's counters: BytesRead / BytesWritten per second (KiB = 1024).
// Then BASELINE cfg1 (RS t=3, block_size 512 -> RS(255,249), 4096 blocks): per-block
// writeBlock/readBlock loops vs one writeBlocks/readBlocks call over the same 4096 blocks.
//
// One line of JSON per case.  Usage: bench_blockdevice [min_seconds_per_case]
#include "ppfs_gpu/block_device.hpp"

#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

using namespace ppfs_gpu;
using clk = std::chrono::steady_clock;

static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

template <class F> static std::pair<double, long> run_for(double min_s, F&& f)
{
    long it = 0;
    const auto t0 = clk::now();
    double el = 0;
    do {
        for (int i = 0; i < 16; ++i, ++it)
            f();
        el = secs(t0, clk::now());
    } while (el < min_s);
    return { el, it };
}

int main(int argc, char** argv)
{
    const double min_s = argc > 1 ? std::atof(argv[1]) : 0.2;
    const size_t block_size = 256;
    // one disk per device (the reference's fixtures each build their own), so a device's blocks
    // 0 and 1 are its own formatted codewords
    std::vector<std::unique_ptr<StackDisk<>>> disks;
    for (int i = 0; i < 4; ++i)
        disks.push_back(std::make_unique<StackDisk<>>());
    RawBlockDevice raw(block_size, *disks[0]);
    ReedSolomonBlockDevice rs(*disks[1], block_size, 16);
    HammingBlockDevice hamming((int)std::log2(block_size), *disks[2]);
    CrcBlockDevice crc(CrcPolynomial::MsgImplicit(0xea), *disks[3], block_size);
    std::map<std::string, IBlockDevice*> devs = { { "raw", &raw }, { "crc", &crc }, { "hamming", &hamming },
        { "rs", &rs } };
    for (auto& kv : devs) // blocks 0 and 1 valid for every codec
        for (unsigned b = 0; b < 2; ++b)
            (void)kv.second->formatBlock(b);

    for (const char* name : { "raw", "crc", "hamming", "rs" }) {
        IBlockDevice& dev = *devs[name];
        for (size_t n = 1; n <= 256; n *= 2) {
            std::array<uint8_t, 4096> rb;
            static_vector<uint8_t> rd(rb.data(), rb.size());
            double bytes = 0;
            bool ok = true;
            auto r = run_for(min_s, [&] {
                auto ret = dev.readBlock({ 0, 0 }, n, rd);
                ok = ok && ret.has_value();
                bytes += rd.size();
            });
            std::printf("{\"bench\": \"BM_BlockDevice_Read/%s_test/%zu\", \"iterations\": %ld, \"us_per_call\": %.2f, "
                        "\"BytesRead_per_s\": %.0f, \"ok\": %s}\n",
                name, n, r.second, r.first / r.second * 1e6, bytes / r.first, ok ? "true" : "false");
        }
        for (size_t n = 1; n <= 256; n *= 2) {
            std::array<uint8_t, 4096> wb;
            std::fill(wb.begin(), wb.begin() + n, uint8_t { 0x55 });
            static_vector<uint8_t> wd(wb.data(), wb.size(), n);
            double bytes = 0;
            bool ok = true;
            auto r = run_for(min_s, [&] {
                auto ret = dev.writeBlock(wd, { 1, 0 });
                ok = ok && ret.has_value();
                if (ret.has_value())
                    bytes += ret.value();
            });
            std::printf("{\"bench\": \"BM_BlockDevice_Write/%s_test/%zu\", \"iterations\": %ld, \"us_per_call\": %.2f, "
                        "\"BytesWritten_per_s\": %.0f, \"ok\": %s}\n",
                name, n, r.second, r.first / r.second * 1e6, bytes / r.first, ok ? "true" : "false");
        }
    }

    // BASELINE cfg1: RS t=3, block_size 512 -> RS(255,249), 4096 blocks
    {
        const size_t NB = 4096;
        StackDisk<21> d2; // 2 MiB >= 4096 * 255
        ReedSolomonBlockDevice dev(d2, 512, 3);
        const size_t ds = dev.dataSize();
        std::vector<uint8_t> pay(NB * ds), out(NB * ds), err(NB);
        for (size_t i = 0; i < pay.size(); ++i)
            pay[i] = (uint8_t)(i * 131 + 7);
        auto t0 = clk::now();
        for (size_t b = 0; b < NB; ++b) {
            static_vector<uint8_t> v(pay.data() + b * ds, ds, ds);
            (void)dev.writeBlock(v, DataLocation((int)b, 0));
        }
        auto t1 = clk::now();
        bool ok = true;
        for (size_t b = 0; b < NB; ++b) {
            static_vector<uint8_t> v(out.data() + b * ds, ds);
            ok = ok && dev.readBlock(DataLocation((int)b, 0), ds, v).has_value();
        }
        auto t2 = clk::now();
        ok = ok && out == pay;
        (void)dev.writeBlocks(0, NB, pay.data(), err.data()); // warm: staging buffers allocated
        (void)dev.readBlocks(0, NB, out.data(), err.data());
        auto t3 = clk::now();
        (void)dev.writeBlocks(0, NB, pay.data(), err.data());
        auto t4 = clk::now();
        (void)dev.readBlocks(0, NB, out.data(), err.data());
        auto t5 = clk::now();
        ok = ok && out == pay;
        std::printf("{\"bench\": \"cfg1 rs255_t3 4096 blocks\", \"per_block_write_blocks_per_s\": %.0f, "
                    "\"per_block_read_blocks_per_s\": %.0f, \"batched_write_blocks_per_s\": %.0f, "
                    "\"batched_read_blocks_per_s\": %.0f, \"ok\": %s}\n",
            NB / secs(t0, t1), NB / secs(t1, t2), NB / secs(t3, t4), NB / secs(t4, t5), ok ? "true" : "false");
    }
    {
        // a file-backed disk image (MappedFileDisk: shared mmap, page-locked when the runtime
        // allows): one writeBlocks / readBlocks / scrub call over 2^20 RS(255,249) blocks in place
        const size_t NB = size_t(1) << 20;
        char path[] = "/tmp/ppfs_bench_XXXXXX";
        const int fd = mkstemp(path);
        if (fd >= 0)
            ::close(fd);
        MappedFileDisk fdisk;
        bool ok = fdisk.create(path, NB * 255).has_value();
        ::unlink(path);
        ReedSolomonBlockDevice dev(fdisk, 512, 3);
        const size_t ds = dev.dataSize();
        std::vector<uint8_t> pay(NB * ds), out(NB * ds), err(NB);
        for (size_t i = 0; i < pay.size(); ++i)
            pay[i] = (uint8_t)(i * 131 + 7);
        (void)dev.writeBlocks(0, NB, pay.data(), err.data()); // warm
        (void)dev.readBlocks(0, NB, out.data(), err.data());
        auto t0 = clk::now();
        ok = ok && dev.writeBlocks(0, NB, pay.data(), err.data()).has_value();
        auto t1 = clk::now();
        ok = ok && dev.readBlocks(0, NB, out.data(), err.data()).has_value();
        auto t2 = clk::now();
        size_t counts[3] = { 0, 0, 0 };
        ok = ok && dev.scrub(0, NB, counts, nullptr).has_value() && counts[0] == NB;
        auto t3 = clk::now();
        ok = ok && out == pay;
        const double gib = 1024.0 * 1024.0 * 1024.0;
        std::printf("{\"bench\": \"MappedFileDisk rs255_t3 %zu blocks\", \"pinned\": %s, "
                    "\"writeBlocks_GiB_per_s\": %.2f, \"readBlocks_GiB_per_s\": %.2f, \"scrub_GiB_per_s\": %.2f, "
                    "\"ok\": %s}\n",
            NB, fdisk.pinned() ? "true" : "false", NB * (ds + 255) / secs(t0, t1) / gib,
            NB * (ds + 255) / secs(t1, t2) / gib, NB * 255 * 2 / secs(t2, t3) / gib, ok ? "true" : "false");
    }
    return 0;
}
