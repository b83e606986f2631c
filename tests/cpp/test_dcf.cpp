// C++ mirror of the reference's own tests (lib.rs:351-443, prg.rs:76-97),
// written against include/dcf.hpp and run on the GPU (tests/test_cpp_mirror.py).
// thread_rng() seeds are replaced by fixed bytes; a golden PRG row pins bits.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>

#include "dcf.hpp"

using Bytes16 = std::array<uint8_t, 16>;
using Key32 = std::array<uint8_t, 32>;

static int failures = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

template <size_t L>
static std::array<uint8_t, L> hex(const char* h) {
  std::array<uint8_t, L> a{};
  for (size_t i = 0; i < L; ++i) a[i] = (uint8_t)std::stoul(std::string(h + 2 * i, 2), nullptr, 16);
  return a;
}

// lib.rs:359-370 (decoded)
static const Key32 KEY0 = hex<32>("6a391b5fb358f333ac57151b0831324bb349b990721c4eb5ee3957d3bb40c664");
static const Key32 KEY1 = hex<32>("9b15c80fb7bc21719e89b8f70ea0539d4efa0c3b16e4988262fc6479b58c7bc2");
static const Bytes16 ALPHAS[5] = {hex<16>("4ba957f5dd05e9fc3f04f6fb556fa843"),
                                  hex<16>("c2474bdac6bb999846712266b78c7355"),
                                  hex<16>("c2474bdac6bb999846712266b78c7356"),
                                  hex<16>("c2474bdac6bb999846712266b78c7357"),
                                  hex<16>("ef9697d78f8aa441500ab335b56bff97")};
static const Bytes16 BETA = hex<16>("03119712438ae92381a8dea88f20c0bb");
static const Bytes16 SEED = hex<16>("2a4c8f2579125a942a458f242b4e4819");  // prg.rs:84

using Prg16 = dcf::Aes256HirosePrg<16, 2>;
using Dcf16 = dcf::DcfImpl<16, 16, Prg16>;

template <class DcfT>
static void eval_both(const DcfT& d, const dcf::Share<16>& k, std::vector<Bytes16>& ys0, std::vector<Bytes16>& ys1) {
  dcf::Share<16> k0 = k, k1 = k;
  k0.s0s = {k.s0s[0]};  // lib.rs:382-385
  k1.s0s = {k.s0s[1]};
  std::vector<const Bytes16*> xs;
  for (auto& a : ALPHAS) xs.push_back(&a);
  ys0.assign(5, Bytes16{});
  ys1.assign(5, Bytes16{});
  std::vector<Bytes16*> y0p, y1p;
  for (int i = 0; i < 5; ++i) {
    y0p.push_back(&ys0[i]);
    y1p.push_back(&ys1[i]);
  }
  d.eval(false, k0, xs, y0p);
  d.eval(true, k1, xs, y1p);
}

template <class PrgT>
static void reconstruction(const PrgT& prg, dcf::BoundState bound, const int expect[5]) {
  dcf::DcfImpl<16, 16, PrgT> d(prg);
  for (int trial = 0; trial < 3; ++trial) {
    Bytes16 s0{}, s1{};
    for (int i = 0; i < 16; ++i) {
      s0[i] = (uint8_t)(17 * i + 3 * trial + 1);
      s1[i] = (uint8_t)(29 * i + 7 * trial + 5);
    }
    dcf::CmpFn<16, 16> f{ALPHAS[2], BETA};
    auto k = d.gen(f, {&s0, &s1}, bound);
    CHECK(k.cws.size() == 128 && k.s0s.size() == 2);
    std::vector<Bytes16> ys0, ys1;
    eval_both(d, k, ys0, ys1);
    for (int i = 0; i < 5; ++i) {
      Bytes16 r{};
      for (int j = 0; j < 16; ++j) r[j] = ys0[i][j] ^ ys1[i][j];
      CHECK(r == (expect[i] ? BETA : Bytes16{}));
    }
    CHECK(ys0[2] != Bytes16{});  // lib.rs:440-441
    CHECK(ys1[2] != Bytes16{});
  }
}

int main() {
  Prg16 prg({&KEY0, &KEY1});
  // The same two reference tests over the MMO PRG (north_star; keys = halves of KEYS).
  std::array<uint8_t, 16> mk[4];
  for (int i = 0; i < 4; ++i) std::memcpy(mk[i].data(), (i < 2 ? KEY0 : KEY1).data() + 16 * (i & 1), 16);
  dcf::Aes128MatyasMeyerOseasPrg<16, 4> mmo({&mk[0], &mk[1], &mk[2], &mk[3]});
  {  // test_dcf_gen_then_eval_ok (lib.rs:372-395)
    const int expect[5] = {1, 1, 0, 0, 0};
    reconstruction(prg, dcf::BoundState::LtBeta, expect);
    reconstruction(mmo, dcf::BoundState::LtBeta, expect);
  }
  {  // test_dcf_gen_gt_beta_then_eval_ok (lib.rs:397-420)
    const int expect[5] = {0, 0, 0, 1, 1};
    reconstruction(prg, dcf::BoundState::GtBeta, expect);
    reconstruction(mmo, dcf::BoundState::GtBeta, expect);
  }
  {  // test_prg_gen_not_zeros (prg.rs:86-96) + golden row (tests/golden/prg16.json rows[0])
    auto out = prg.gen(SEED);
    for (int i = 0; i < 2; ++i) {
      CHECK(std::get<0>(out[i]) != Bytes16{});
      CHECK(std::get<1>(out[i]) != Bytes16{});
    }
    const char* want = std::getenv("DCF_PRG16_ROW0_SL");
    if (want) CHECK(std::get<0>(out[0]) == hex<16>(want));
  }
  {  // panics of the reference become exceptions
    Dcf16 d(prg);
    Bytes16 s0{}, s1{};
    auto k = d.gen(dcf::CmpFn<16, 16>{ALPHAS[0], BETA}, {&s0, &s1}, dcf::BoundState::LtBeta);
    k.cws.pop_back();
    bool threw = false;
    try {
      std::vector<const Bytes16*> xs{&ALPHAS[0]};
      Bytes16 y{};
      d.eval(false, k, xs, {&y});
    } catch (const dcf::Error& e) {
      threw = e.code() == DCF_ERR_KEY;
    }
    CHECK(threw);
    threw = false;
    try {
      Key32 z{};
      std::array<const Key32*, 17> ks;
      ks.fill(&z);
      dcf::Aes256HirosePrg<32, 17> bad(ks);  // prg.rs:51 would index ciphers[17]
    } catch (const dcf::Error& e) {
      threw = e.code() == DCF_ERR_CIPHER_N;
    }
    CHECK(threw);
  }
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "cpp mirror ok", failures);
  return failures ? 1 : 0;
}
