// dcf.hpp — C++17 host mirror of the `dcf` crate's operator / plugin interface
// (xymeng16/dcf v0.2.2), running on MI355X through the C ABI of dcf_hip.h.
//
//   Rust (reference)                                  C++ (here)
//   trait Dcf<N, LAMBDA> { gen, eval }  lib.rs:24-35  dcf::Dcf<N, LAMBDA>
//   struct CmpFn { alpha, beta }        lib.rs:41-46  dcf::CmpFn<N, LAMBDA>
//   trait Prg<LAMBDA>                   lib.rs:52-54  dcf::Prg<LAMBDA> (concept-like base)
//   Aes256HirosePrg<LAMBDA, CIPHER_N>   prg.rs:22-33  dcf::Aes256HirosePrg<LAMBDA, CIPHER_N>
//   DcfImpl<N, LAMBDA, PrgT>::new(prg)  lib.rs:63-77  dcf::DcfImpl<N, LAMBDA, PrgT>(prg)
//   struct Cw { s, v, tl, tr }          lib.rs:209    dcf::Cw<LAMBDA>
//   struct Share { s0s, cws, cw_np1 }   lib.rs:275    dcf::Share<LAMBDA>
//   enum BoundState { LtBeta, GtBeta }  lib.rs:342    dcf::BoundState
//
// Same argument meaning: `eval(b, k, xs, ys)` evaluates party b with seed
// k.s0s[0] (lib.rs:168) and overwrites ys (lib.rs:171).  Where the reference
// panics (k.cws.len() != 8N, lib.rs:165; cipher index, prg.rs:51) this throws
// dcf::Error; where it silently truncates (xs.len() != ys.len(), lib.rs:196)
// this throws too.  All compute runs in libdcf_hip.so on the GPU.
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "dcf_hip.h"

namespace dcf {

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& msg) : std::runtime_error(msg), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline void check(int rc) {
  if (rc != DCF_OK) throw Error(rc, std::string("dcf_hip: ") + dcf_last_error());
}

enum class BoundState : int { LtBeta = DCF_BOUND_LT_BETA, GtBeta = DCF_BOUND_GT_BETA };

template <size_t N, size_t LAMBDA>
struct CmpFn {
  std::array<uint8_t, N> alpha;
  std::array<uint8_t, LAMBDA> beta;
};

template <size_t LAMBDA>
struct Cw {
  std::array<uint8_t, LAMBDA> s;
  std::array<uint8_t, LAMBDA> v;
  bool tl;
  bool tr;
  bool operator==(const Cw& o) const { return s == o.s && v == o.v && tl == o.tl && tr == o.tr; }
};

template <size_t LAMBDA>
struct Share {
  std::vector<std::array<uint8_t, LAMBDA>> s0s;  // gen: 2 entries; eval reads s0s[0]
  std::vector<Cw<LAMBDA>> cws;                   // 8 * N entries
  std::array<uint8_t, LAMBDA> cw_np1;
};

template <size_t LAMBDA>
using PrgOut = std::array<std::tuple<std::array<uint8_t, LAMBDA>, std::array<uint8_t, LAMBDA>, bool>, 2>;

// `Prg<LAMBDA>` (lib.rs:52-54): seed -> [(s_l, v_l, t_l), (s_r, v_r, t_r)].
template <size_t LAMBDA>
class Prg {
 public:
  virtual ~Prg() = default;
  virtual PrgOut<LAMBDA> gen(const std::array<uint8_t, LAMBDA>& seed) const = 0;
  virtual dcf_prg* handle() const = 0;
};

// Aes256HirosePrg<LAMBDA, CIPHER_N>::new(keys) (prg.rs:27-33), resident on `device`.
template <size_t LAMBDA, size_t CIPHER_N>
class Aes256HirosePrg final : public Prg<LAMBDA> {
 public:
  explicit Aes256HirosePrg(const std::array<const std::array<uint8_t, 32>*, CIPHER_N>& keys, int device = 0) {
    std::vector<uint8_t> blob(32 * CIPHER_N);
    for (size_t i = 0; i < CIPHER_N; ++i) std::memcpy(blob.data() + 32 * i, keys[i]->data(), 32);
    check(dcf_hirose_prg_new(blob.data(), CIPHER_N, LAMBDA, device, &h_));
  }
  ~Aes256HirosePrg() override { dcf_prg_free(h_); }
  Aes256HirosePrg(const Aes256HirosePrg&) = delete;
  Aes256HirosePrg& operator=(const Aes256HirosePrg&) = delete;
  Aes256HirosePrg(Aes256HirosePrg&& o) noexcept : h_(o.h_) { o.h_ = nullptr; }

  PrgOut<LAMBDA> gen(const std::array<uint8_t, LAMBDA>& seed) const override {
    std::vector<uint8_t> out(4 * LAMBDA + 2);
    check(dcf_prg_gen(h_, seed.data(), 1, out.data()));
    PrgOut<LAMBDA> r;
    auto slice = [&](size_t i) {
      std::array<uint8_t, LAMBDA> a;
      std::memcpy(a.data(), out.data() + i * LAMBDA, LAMBDA);
      return a;
    };
    r[0] = std::make_tuple(slice(0), slice(1), out[4 * LAMBDA] != 0);
    r[1] = std::make_tuple(slice(2), slice(3), out[4 * LAMBDA + 1] != 0);
    return r;
  }
  dcf_prg* handle() const override { return h_; }

 private:
  dcf_prg* h_ = nullptr;
};

// Aes128MatyasMeyerOseasPrg<LAMBDA, CIPHER_N>::new(keys): the PRG BASELINE.json's
// north_star names (not in the reference crate; definition in dcf_hip.h,
// dcf_mmo_prg_new; parity unpinned).  CIPHER_N >= 4 AES-128 keys, LAMBDA = 16.
template <size_t LAMBDA, size_t CIPHER_N>
class Aes128MatyasMeyerOseasPrg final : public Prg<LAMBDA> {
 public:
  explicit Aes128MatyasMeyerOseasPrg(const std::array<const std::array<uint8_t, 16>*, CIPHER_N>& keys,
                                     int device = 0) {
    std::vector<uint8_t> blob(16 * CIPHER_N);
    for (size_t i = 0; i < CIPHER_N; ++i) std::memcpy(blob.data() + 16 * i, keys[i]->data(), 16);
    check(dcf_mmo_prg_new(blob.data(), CIPHER_N, LAMBDA, device, &h_));
  }
  ~Aes128MatyasMeyerOseasPrg() override { dcf_prg_free(h_); }
  Aes128MatyasMeyerOseasPrg(const Aes128MatyasMeyerOseasPrg&) = delete;
  Aes128MatyasMeyerOseasPrg& operator=(const Aes128MatyasMeyerOseasPrg&) = delete;

  PrgOut<LAMBDA> gen(const std::array<uint8_t, LAMBDA>& seed) const override {
    std::vector<uint8_t> out(4 * LAMBDA + 2);
    check(dcf_prg_gen(h_, seed.data(), 1, out.data()));
    PrgOut<LAMBDA> r;
    auto slice = [&](size_t i) {
      std::array<uint8_t, LAMBDA> a;
      std::memcpy(a.data(), out.data() + i * LAMBDA, LAMBDA);
      return a;
    };
    r[0] = std::make_tuple(slice(0), slice(1), out[4 * LAMBDA] != 0);
    r[1] = std::make_tuple(slice(2), slice(3), out[4 * LAMBDA + 1] != 0);
    return r;
  }
  dcf_prg* handle() const override { return h_; }

 private:
  dcf_prg* h_ = nullptr;
};

// `Dcf<N, LAMBDA>` (lib.rs:24-35).
template <size_t N, size_t LAMBDA>
class Dcf {
 public:
  virtual ~Dcf() = default;
  virtual Share<LAMBDA> gen(const CmpFn<N, LAMBDA>& f, const std::array<const std::array<uint8_t, LAMBDA>*, 2>& s0s,
                            BoundState bound) const = 0;
  virtual void eval(bool b, const Share<LAMBDA>& k, const std::vector<const std::array<uint8_t, N>*>& xs,
                    const std::vector<std::array<uint8_t, LAMBDA>*>& ys) const = 0;
};

// Single-key correction-word block (layout in dcf_hip.h).
template <size_t N, size_t LAMBDA>
std::vector<uint8_t> share_to_cwb(const Share<LAMBDA>& k) {
  constexpr size_t n = 8 * N;
  if (k.cws.size() != n)
    throw Error(DCF_ERR_KEY, "k.cws.len() != N * 8 (lib.rs:165)");
  std::vector<uint8_t> cwb(dcf_cwb_bytes(N, LAMBDA, 1), 0);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(cwb.data() + i * LAMBDA, k.cws[i].s.data(), LAMBDA);
    std::memcpy(cwb.data() + (n + i) * LAMBDA, k.cws[i].v.data(), LAMBDA);
    cwb[2 * n * LAMBDA + i] = (uint8_t)((k.cws[i].tl ? 1 : 0) | (k.cws[i].tr ? 2 : 0));
  }
  std::memcpy(cwb.data() + dcf_cwb_np1_offset(N, LAMBDA, 1), k.cw_np1.data(), LAMBDA);
  return cwb;
}

template <size_t N, size_t LAMBDA>
Share<LAMBDA> cwb_to_share(const std::vector<uint8_t>& cwb, std::vector<std::array<uint8_t, LAMBDA>> s0s) {
  constexpr size_t n = 8 * N;
  Share<LAMBDA> k;
  k.s0s = std::move(s0s);
  k.cws.resize(n);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(k.cws[i].s.data(), cwb.data() + i * LAMBDA, LAMBDA);
    std::memcpy(k.cws[i].v.data(), cwb.data() + (n + i) * LAMBDA, LAMBDA);
    k.cws[i].tl = (cwb[2 * n * LAMBDA + i] & 1) != 0;
    k.cws[i].tr = (cwb[2 * n * LAMBDA + i] & 2) != 0;
  }
  std::memcpy(k.cw_np1.data(), cwb.data() + dcf_cwb_np1_offset(N, LAMBDA, 1), LAMBDA);
  return k;
}

// DcfImpl<N, LAMBDA, PrgT> (lib.rs:63-205) on the GPU.
template <size_t N, size_t LAMBDA, class PrgT>
class DcfImpl final : public Dcf<N, LAMBDA> {
 public:
  explicit DcfImpl(const PrgT& prg) : prg_(prg) {}

  Share<LAMBDA> gen(const CmpFn<N, LAMBDA>& f, const std::array<const std::array<uint8_t, LAMBDA>*, 2>& s0s,
                    BoundState bound) const override {
    std::vector<uint8_t> cwb(dcf_cwb_bytes(N, LAMBDA, 1));
    check(dcf_gen(prg_.handle(), N, f.alpha.data(), f.beta.data(), s0s[0]->data(), s0s[1]->data(), (int)bound,
                  cwb.data()));
    return cwb_to_share<N, LAMBDA>(cwb, {*s0s[0], *s0s[1]});
  }

  void eval(bool b, const Share<LAMBDA>& k, const std::vector<const std::array<uint8_t, N>*>& xs,
            const std::vector<std::array<uint8_t, LAMBDA>*>& ys) const override {
    if (xs.size() != ys.size()) throw Error(DCF_ERR_LEN, "xs.len() != ys.len() (lib.rs:196 would truncate)");
    std::vector<uint8_t> xbuf(xs.size() * N), ybuf(ys.size() * LAMBDA);
    for (size_t i = 0; i < xs.size(); ++i) std::memcpy(xbuf.data() + i * N, xs[i]->data(), N);
    eval_contiguous(b, k, xbuf.data(), xs.size(), ybuf.data());
    for (size_t i = 0; i < ys.size(); ++i) std::memcpy(ys[i]->data(), ybuf.data() + i * LAMBDA, LAMBDA);
  }

  // Contiguous form: xs = m * N bytes, ys = m * LAMBDA bytes.
  void eval_contiguous(bool b, const Share<LAMBDA>& k, const uint8_t* xs, size_t m, uint8_t* ys) const {
    if (k.s0s.empty()) throw Error(DCF_ERR_KEY, "k.s0s is empty (lib.rs:168 reads s0s[0])");
    const std::vector<uint8_t> cwb = share_to_cwb<N, LAMBDA>(k);
    check(dcf_eval(prg_.handle(), N, b ? 1 : 0, cwb.data(), cwb.size(), k.s0s[0].data(), xs, m, ys, m * LAMBDA));
  }

 private:
  const PrgT& prg_;
};

}  // namespace dcf
