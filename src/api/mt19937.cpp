// MT19937 Mersenne Twister (Matsumoto & Nishimura 1998), the generator the
// reference seeds and draws measurement outcomes from (QuEST/src/mt19937ar.c:
// init_by_array :80, genrand_real1 :150).  Re-implemented here; the output
// sequence is bit-identical to the canonical algorithm, which the golden test
// tests/test_reference_suite.py::test_seed_quest_mt19937_golden pins
// (seedQuEST.test:9-15 in the reference).
//
// One generator per process; every rank seeds it identically, so all ranks
// draw the same measurement outcome without communicating.
#include <cstdint>

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;

struct MT {
    uint32_t s[kN];
    int idx = kN + 1;  // kN+1: not yet seeded

    void seed(uint32_t v) {
        s[0] = v;
        for (int i = 1; i < kN; i++) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + (uint32_t)i;
        idx = kN;
    }

    // 64-bit key words are folded exactly as the canonical C code does with
    // `unsigned long` arithmetic followed by a 32-bit mask.
    void seedArray(const unsigned long* key, int len) {
        seed(19650218u);
        int i = 1, j = 0;
        for (int k = (kN > len ? kN : len); k > 0; k--) {
            unsigned long prev = s[i - 1];
            unsigned long v = ((unsigned long)s[i] ^ ((prev ^ (prev >> 30)) * 1664525ul)) + key[j] + (unsigned long)j;
            s[i] = (uint32_t)(v & 0xffffffffUL);
            if (++i >= kN) {
                s[0] = s[kN - 1];
                i = 1;
            }
            if (++j >= len) j = 0;
        }
        for (int k = kN - 1; k > 0; k--) {
            unsigned long prev = s[i - 1];
            unsigned long v = ((unsigned long)s[i] ^ ((prev ^ (prev >> 30)) * 1566083941ul)) - (unsigned long)i;
            s[i] = (uint32_t)(v & 0xffffffffUL);
            if (++i >= kN) {
                s[0] = s[kN - 1];
                i = 1;
            }
        }
        s[0] = 0x80000000u;
        idx = kN;
    }

    void twist() {
        for (int k = 0; k < kN; k++) {
            uint32_t y = (s[k] & kUpper) | (s[(k + 1) % kN] & kLower);
            s[k] = s[(k + kM) % kN] ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
        }
        idx = 0;
    }

    uint32_t next() {
        if (idx >= kN) {
            if (idx == kN + 1) seed(5489u);
            twist();
        }
        uint32_t y = s[idx++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
};

MT g_mt;

}  // namespace

extern "C" {

void init_genrand(unsigned long s) { g_mt.seed((uint32_t)(s & 0xffffffffUL)); }
void init_by_array(unsigned long init_key[], int key_length) { g_mt.seedArray(init_key, key_length); }
unsigned long genrand_int32(void) { return g_mt.next(); }
long genrand_int31(void) { return (long)(g_mt.next() >> 1); }
// [0,1]
double genrand_real1(void) { return g_mt.next() * (1.0 / 4294967295.0); }
// [0,1)
double genrand_real2(void) { return g_mt.next() * (1.0 / 4294967296.0); }
// (0,1)
double genrand_real3(void) { return ((double)g_mt.next() + 0.5) * (1.0 / 4294967296.0); }
// [0,1) with 53-bit resolution
double genrand_res53(void) {
    unsigned long a = g_mt.next() >> 5, b = g_mt.next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}
}
