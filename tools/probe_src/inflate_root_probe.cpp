// Literal-table root size vs decode rate on fp32 weights (tools/inflate_root_probe.sh builds one
// binary per root; run on the box). Not part of the product build.
#include "../../fedn_amd/csrc/inflate.h"
#include <zlib.h>
#include <chrono>
#include <cstdio>
#include <memory>
#include <random>
#include <vector>
int main() {
    std::mt19937_64 rng(1);
    std::normal_distribution<float> nd;
    const size_t n = 100000000;
    std::vector<uint8_t> b(n);
    for (size_t i = 0; i + 4 <= n; i += 4) { float f = nd(rng); std::memcpy(&b[i], &f, 4); }
    z_stream zs{};
    deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    std::vector<uint8_t> cb(n + n / 8 + 1024);
    zs.next_in = b.data(); zs.avail_in = (uInt)n; zs.next_out = cb.data(); zs.avail_out = (uInt)cb.size();
    deflate(&zs, Z_FINISH); cb.resize(zs.total_out); deflateEnd(&zs);
    std::vector<uint8_t> out(n);
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
        auto t1 = std::chrono::steady_clock::now();
        std::unique_ptr<fnpz_fast::Inflate> dec(new fnpz_fast::Inflate(cb.data(), cb.size()));
        uint8_t* o = out.data();
        dec->run(&o, out.data() + n, out.data());
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    }
    std::printf("{\"root\": %d, \"MBps\": %.0f, \"same\": %d}\n", FNPZ_LIT_ROOT, n / best / 1e6, std::memcmp(out.data(), b.data(), n) == 0);
}
