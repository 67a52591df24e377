#pragma once
// server_box.hpp -- mailbox of the resident small-batch server (rs_wg.hpp rs_wg_server_kernel,
// api.cpp server_call).  One per engine context, in host-coherent memory mapped to the device.
//
// Protocol.  The host writes the request's input bytes into the context's zero-copy buffer (the
// srv_layout offsets) and then the whole request as ONE 32-bit word, `cmd` (release store):
// sequence number, op, write-back, want-data and the block count.  The resident workgroup's lane 0
// polls `cmd` and `stop` with one 8-byte relaxed system-scope load per poll (one PCIe round trip,
// s_sleep between polls), so a request can never be seen half-written.  On a new `cmd` the
// workgroup runs it, makes its stores visible system-wide and stores `done` = cmd (release); the
// host spins on `done`.  `alive` = the launch generation while the kernel polls and generation |
// SRV_EXITED once it has returned: it leaves on `stop`, after idle_us without a request, or after
// SRV_LIFETIME_US in any case, so a launch never outlives a burst of per-block calls by much (a
// device-wide synchronize waits for it) and the host relaunches it on demand.
#include <stdint.h>

namespace ppfs {

enum : uint32_t { SRV_ENCODE = 0, SRV_DECODE = 1, SRV_WRITE = 2 };
constexpr uint32_t SRV_EXITED = 0x80000000u;
// One launch serves at most 20 ms.  HIP maps a process's streams onto GPU_MAX_HW_QUEUES (4) hardware
// queues, so another stream (another context's, the caller's) can sit behind the resident launch on
// its queue: the lifetime bounds that wait (round 3: 1 s stalled a second context's creation and
// first copies for seconds while the first one served per-block calls).  A relaunch costs ~10 us.
constexpr uint64_t SRV_LIFETIME_US = 20000;
constexpr uint32_t SRV_MAX_BLOCKS = 64;

// cmd word: bits 0-6 block count (1..64), 12-13 op, 14 write-back, 15 want data, 16-31 sequence
struct SrvCmd {
    uint32_t nb, op;
    bool write_back, want_data;
};
inline constexpr uint32_t srv_cmd_pack(uint32_t seq, const SrvCmd& c)
{
    return (seq << 16) | (c.want_data ? 1u << 15 : 0u) | (c.write_back ? 1u << 14 : 0u) | ((c.op & 3u) << 12)
        | (c.nb & 0x7Fu);
}
inline constexpr SrvCmd srv_cmd_unpack(uint32_t w)
{
    return SrvCmd { w & 0x7Fu, (w >> 12) & 3u, ((w >> 14) & 1u) != 0, ((w >> 15) & 1u) != 0 };
}

// offsets of a request's buffers in the zero-copy buffer (api.cpp layout_for: same 256-byte rounding)
struct SrvLayout {
    uint32_t data, raw, status;
};
inline constexpr uint32_t srv_al(uint32_t x) { return (x + 255u) & ~255u; }
inline constexpr SrvLayout srv_layout(uint32_t nb, uint32_t k, uint32_t n)
{
    return SrvLayout { 0u, srv_al(nb * k), srv_al(srv_al(nb * k) + nb * n) };
}

struct alignas(64) SrvBox {
    uint32_t cmd;  // host -> device: the request (one word)
    uint32_t stop; // host -> device: leave now
    uint32_t pad0[14];
    uint32_t done;   // device -> host: the last cmd served
    uint32_t alive;  // device -> host: generation (| SRV_EXITED after return)
    uint64_t served; // requests served by this launch (diagnostics)
    uint32_t flag;   // device -> host: completion of the launch path (api.cpp wait_flag)
    uint32_t pad1[11];
};
static_assert(sizeof(SrvBox) == 128, "mailbox layout: one request line, one reply line");

} // namespace ppfs
