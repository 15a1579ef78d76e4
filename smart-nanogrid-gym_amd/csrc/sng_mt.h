// sng_mt.h -- host MT19937 streams with the exact draw semantics of the two global RNGs the
// reference consumes in reset()/step():
//   numpy legacy RandomState (np.random.seed / rand / uniform / randint), used by
//     ChargingStation.generate_initial_vehicle_presence_per_charger (charging_station.py:200-279)
//   Python `random` (random.seed / randint), used for random_pv_shift_ratio
//     (smart_nanogrid_environment.py:181, 349)
#pragma once
#include <stdint.h>

namespace sng {

class MT19937 {
   public:
    static constexpr int N = 624, M = 397;

    // np.random.seed(int): numpy's legacy seeding is init_genrand(seed & 0xffffffff)
    void seed_numpy(uint32_t s) { init_genrand(s); }

    // random.seed(int): init_by_array over the little-endian 32-bit words of |seed|
    void seed_python(uint64_t s) {
        uint32_t key[2];
        int len = 0;
        do {
            key[len++] = (uint32_t)(s & 0xffffffffu);
            s >>= 32;
        } while (s && len < 2);
        init_by_array(key, len);
    }

    uint32_t next() {
        if (mti_ >= N) twist();
        uint32_t y = mt_[mti_++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }

    // numpy random_sample(): (a >> 5, b >> 6) -> 53-bit double in [0, 1)
    double random() {
        const int32_t a = (int32_t)(next() >> 5), b = (int32_t)(next() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }

    // numpy legacy uniform(low, high) = low + (high - low) * random_sample()
    double uniform(double low, double high) {
        const double range = high - low;
        return low + range * random();
    }

    // numpy legacy randint(low, high), int64, exclusive high: masked rejection on 32-bit
    // draws (random_bounded_uint64_fill, use_masked=True); a one-value range draws nothing.
    int64_t randint(int64_t low, int64_t high) {
        const uint64_t rng = (uint64_t)(high - 1 - low);
        if (rng == 0) return low;
        uint64_t mask = rng;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        mask |= mask >> 32;
        uint32_t v;
        while ((v = (next() & (uint32_t)mask)) > (uint32_t)rng) {
        }
        return low + (int64_t)v;
    }

    // Python random.randint(a, b): a + _randbelow(b - a + 1) via getrandbits(bit_length)
    int64_t py_randint(int64_t a, int64_t b) {
        const uint64_t n = (uint64_t)(b - a + 1);
        int k = 0;
        while (k < 64 && (n >> k) != 0) ++k;
        uint32_t r;
        do {
            r = next() >> (32 - k);
        } while (r >= n);
        return a + (int64_t)r;
    }

    // checkpoint / resume (sng_get_state): the 624 state words and the position
    // prefetch targets of the next draw (the host ratio draws walk tens of thousands of streams)
    const void *pos_addr() const { return &mti_; }
    const void *next_addr() const { return &mt_[mti_ < N ? mti_ : 0]; }
    static constexpr int kStateWords = N + 1;
    void save(uint32_t *out) const {
        for (int i = 0; i < N; ++i) out[i] = mt_[i];
        out[N] = (uint32_t)mti_;
    }
    bool load(const uint32_t *in) {
        if (in[N] > (uint32_t)N + 1) return false;
        for (int i = 0; i < N; ++i) mt_[i] = in[i];
        mti_ = (int)in[N];
        return true;
    }

   private:
    uint32_t mt_[N];
    int mti_ = N + 1;

    void init_genrand(uint32_t s) {
        mt_[0] = s;
        for (int i = 1; i < N; ++i) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
        mti_ = N;
    }

    void init_by_array(const uint32_t *key, int len) {
        init_genrand(19650218u);
        int i = 1, j = 0;
        for (int k = (N > len ? N : len); k; --k) {
            mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            ++i;
            ++j;
            if (i >= N) {
                mt_[0] = mt_[N - 1];
                i = 1;
            }
            if (j >= len) j = 0;
        }
        for (int k = N - 1; k; --k) {
            mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            ++i;
            if (i >= N) {
                mt_[0] = mt_[N - 1];
                i = 1;
            }
        }
        mt_[0] = 0x80000000u;
        mti_ = N;
    }

    void twist() {
        static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
        int kk = 0;
        uint32_t y;
        for (; kk < N - M; ++kk) {
            y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
            mt_[kk] = mt_[kk + M] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < N - 1; ++kk) {
            y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
            mt_[kk] = mt_[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (mt_[N - 1] & 0x80000000u) | (mt_[0] & 0x7fffffffu);
        mt_[N - 1] = mt_[M - 1] ^ (y >> 1) ^ mag01[y & 1u];
        mti_ = 0;
    }
};

}  // namespace sng
