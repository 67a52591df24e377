// ref_gf256_harness.cpp -- TEST INFRASTRUCTURE ONLY.  Exposes the REFERENCE's own GF256 class
// (lib/ecc_helpers/src/gf256.cpp, compiled unmodified from /root/reference by oracle/Makefile into
// oracle/_ref/) through a C ABI, so the oracle's GF(2^8) restatement can be pinned exhaustively
// against the reference binary: every product, quotient (including the a/0 = 0 rule,
// gf256.cpp:56-64), inverse (inv(0) = 0, :76-81) and logarithm (:72).  Nothing in the product path
// or on the GPU box loads this library.
#include <cstddef>
#include <cstdint>

#include "ppfs/ecc_helpers/gf256.hpp"

extern "C" {

// mul / div: 256 x 256 tables indexed [a * 256 + b]; inv, log: 256 entries;
// pow: alpha^i for i = 0..255 by repeated multiplication with getPrimitiveElement()
__attribute__((visibility("default"))) void ref_gf256_dump(uint8_t* mul, uint8_t* div, uint8_t* inv, uint8_t* log,
    uint8_t* pow)
{
    for (int a = 0; a < 256; ++a) {
        const GF256 x(static_cast<uint8_t>(a));
        for (int b = 0; b < 256; ++b) {
            const GF256 y(static_cast<uint8_t>(b));
            mul[a * 256 + b] = static_cast<uint8_t>(x * y);
            div[a * 256 + b] = static_cast<uint8_t>(x / y);
        }
        inv[a] = static_cast<uint8_t>(x.inv());
        log[a] = x.log();
    }
    GF256 p(1);
    for (int i = 0; i < 256; ++i) {
        pow[i] = static_cast<uint8_t>(p);
        p = p * GF256::getPrimitiveElement();
    }
}

// additive group: + and - are XOR (gf256.cpp:42-44); returns the number of pairs that differ
__attribute__((visibility("default"))) int ref_gf256_add_mismatches(void)
{
    int bad = 0;
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b) {
            const GF256 x(static_cast<uint8_t>(a)), y(static_cast<uint8_t>(b));
            bad += static_cast<uint8_t>(x + y) != (a ^ b);
            bad += static_cast<uint8_t>(x - y) != (a ^ b);
            bad += static_cast<uint8_t>(-x) != a;
        }
    return bad;
}
}
