//! `dcf-hip`: the `dcf` crate's [`Dcf`] trait (lib.rs:24-35 of xymeng16/dcf) on MI355X.
//!
//! A caller of `DcfImpl::<N, LAMBDA, _>::new(Aes256HirosePrg::new(keys))` switches by
//! constructing [`DcfHip::<N, LAMBDA>::new(keys, device)`]; `gen` / `eval` keep their
//! signatures and bytes (bit-exact with the CPU restatement of the crate, see the repo's
//! tests).  [`DcfHipMulti`] spreads one `eval` over several GPUs of the node, as the
//! crate spreads it over host cores with rayon (lib.rs:194-199).
//!
//! Errors: the crate panics on a malformed key (lib.rs:165) and on too few ciphers
//! (prg.rs:51); so does this shim (with the library's message), keeping the trait's
//! infallible signatures.  The `try_*` methods return the status instead.
//!
//! NOT compiled in the build container (no Rust toolchain); see INTEGRATION.md.
pub mod ffi;

use std::ffi::CStr;
use std::os::raw::c_int;

use dcf::{BoundState, CmpFn, Cw, Dcf, Share};

/// A non-zero status of the C ABI with the library's message (`dcf_last_error`).
#[derive(Debug, Clone)]
pub struct DcfHipError {
    pub code: c_int,
    pub msg: String,
}

fn check(rc: c_int) -> Result<(), DcfHipError> {
    if rc == ffi::DCF_OK {
        return Ok(());
    }
    let msg = unsafe { CStr::from_ptr(ffi::dcf_last_error()) }.to_string_lossy().into_owned();
    Err(DcfHipError { code: rc, msg })
}

fn bound_code(b: &BoundState) -> c_int {
    match b {
        BoundState::LtBeta => 0,
        BoundState::GtBeta => 1,
    }
}

/// `Share` -> the single-key correction-word block of include/dcf_hip.h.
pub fn share_to_cwb<const N: usize, const LAMBDA: usize>(k: &Share<LAMBDA>) -> Vec<u8> {
    let n = 8 * N;
    assert_eq!(k.cws.len(), n); // lib.rs:165
    let mut b = vec![0u8; unsafe { ffi::dcf_cwb_bytes(N, LAMBDA, 1) }];
    for (i, cw) in k.cws.iter().enumerate() {
        b[i * LAMBDA..(i + 1) * LAMBDA].copy_from_slice(&cw.s);
        b[(n + i) * LAMBDA..(n + i + 1) * LAMBDA].copy_from_slice(&cw.v);
        b[2 * n * LAMBDA + i] = (cw.tl as u8) | ((cw.tr as u8) << 1);
    }
    let off = unsafe { ffi::dcf_cwb_np1_offset(N, LAMBDA, 1) };
    b[off..off + LAMBDA].copy_from_slice(&k.cw_np1);
    b
}

/// The single-key CWB -> `Share { s0s, cws, cw_np1 }`.
pub fn cwb_to_share<const N: usize, const LAMBDA: usize>(b: &[u8], s0s: Vec<[u8; LAMBDA]>) -> Share<LAMBDA> {
    let n = 8 * N;
    let cws = (0..n)
        .map(|i| Cw {
            s: b[i * LAMBDA..(i + 1) * LAMBDA].try_into().unwrap(),
            v: b[(n + i) * LAMBDA..(n + i + 1) * LAMBDA].try_into().unwrap(),
            tl: b[2 * n * LAMBDA + i] & 1 != 0,
            tr: b[2 * n * LAMBDA + i] & 2 != 0,
        })
        .collect();
    let off = unsafe { ffi::dcf_cwb_np1_offset(N, LAMBDA, 1) };
    Share { s0s, cws, cw_np1: b[off..off + LAMBDA].try_into().unwrap() }
}

/// `DcfImpl<N, LAMBDA, Aes256HirosePrg<LAMBDA, CIPHER_N>>` (or the MMO PRG) resident on one GPU.
pub struct DcfHip<const N: usize, const LAMBDA: usize> {
    prg: *mut ffi::DcfPrg,
}

unsafe impl<const N: usize, const LAMBDA: usize> Send for DcfHip<N, LAMBDA> {}
// One dcf_prg may be driven from many threads at once (include/dcf_hip.h "Threading": every
// call leases its own workspace from the prg's pool), as `DcfImpl` is with a `Sync` PRG
// (lib.rs:34,52): an `Arc<DcfHip>` can be shared across rayon or std threads unchanged.
unsafe impl<const N: usize, const LAMBDA: usize> Sync for DcfHip<N, LAMBDA> {}

impl<const N: usize, const LAMBDA: usize> DcfHip<N, LAMBDA> {
    /// `Aes256HirosePrg::<LAMBDA, CIPHER_N>::new(keys)` (prg.rs:27-33) on `device`.
    pub fn new<const CIPHER_N: usize>(keys: [&[u8; 32]; CIPHER_N], device: i32) -> Self {
        Self::try_new(&keys, device).unwrap_or_else(|e| panic!("dcf_hirose_prg_new: {e:?}"))
    }

    pub fn try_new(keys: &[&[u8; 32]], device: i32) -> Result<Self, DcfHipError> {
        let blob: Vec<u8> = keys.iter().flat_map(|k| k.iter().copied()).collect();
        let mut prg = std::ptr::null_mut();
        check(unsafe { ffi::dcf_hirose_prg_new(blob.as_ptr(), keys.len(), LAMBDA, device, &mut prg) })?;
        Ok(Self { prg })
    }

    /// `Aes128MatyasMeyerOseasPrg` (BASELINE.json's north_star PRG; not in the crate):
    /// 4 * LAMBDA / 16 AES-128 keys.
    pub fn new_mmo(keys: &[&[u8; 16]], device: i32) -> Result<Self, DcfHipError> {
        let blob: Vec<u8> = keys.iter().flat_map(|k| k.iter().copied()).collect();
        let mut prg = std::ptr::null_mut();
        check(unsafe { ffi::dcf_mmo_prg_new(blob.as_ptr(), keys.len(), LAMBDA, device, &mut prg) })?;
        Ok(Self { prg })
    }

    pub fn raw(&self) -> *mut ffi::DcfPrg {
        self.prg
    }

    pub fn try_gen(&self, f: &CmpFn<N, LAMBDA>, s0s: [&[u8; LAMBDA]; 2], bound: BoundState)
                   -> Result<Share<LAMBDA>, DcfHipError> {
        let mut b = vec![0u8; unsafe { ffi::dcf_cwb_bytes(N, LAMBDA, 1) }];
        check(unsafe {
            ffi::dcf_gen(self.prg, N, f.alpha.as_ptr(), f.beta.as_ptr(), s0s[0].as_ptr(), s0s[1].as_ptr(),
                         bound_code(&bound), b.as_mut_ptr())
        })?;
        Ok(cwb_to_share::<N, LAMBDA>(&b, vec![*s0s[0], *s0s[1]]))
    }

    pub fn try_eval(&self, b: bool, k: &Share<LAMBDA>, xs: &[&[u8; N]], ys: &mut [&mut [u8; LAMBDA]])
                    -> Result<(), DcfHipError> {
        if xs.len() != ys.len() {
            // the crate zips (lib.rs:196) and silently truncates; the ABI rejects a mismatch
            return Err(DcfHipError { code: ffi::DCF_ERR_LEN, msg: "xs.len() != ys.len()".into() });
        }
        let cwb = share_to_cwb::<N, LAMBDA>(k);
        let xb: Vec<u8> = xs.iter().flat_map(|x| x.iter().copied()).collect();
        let mut yb = vec![0u8; ys.len() * LAMBDA];
        check(unsafe {
            ffi::dcf_eval(self.prg, N, b as c_int, cwb.as_ptr(), cwb.len(), k.s0s[0].as_ptr(), xb.as_ptr(),
                          xs.len(), yb.as_mut_ptr(), yb.len())
        })?;
        for (y, c) in ys.iter_mut().zip(yb.chunks_exact(LAMBDA)) {
            y.copy_from_slice(c);
        }
        Ok(())
    }
}

impl<const N: usize, const LAMBDA: usize> Dcf<N, LAMBDA> for DcfHip<N, LAMBDA> {
    fn gen(&self, f: &CmpFn<N, LAMBDA>, s0s: [&[u8; LAMBDA]; 2], bound: BoundState) -> Share<LAMBDA> {
        self.try_gen(f, s0s, bound).unwrap_or_else(|e| panic!("dcf_gen: {e:?}"))
    }

    fn eval(&self, b: bool, k: &Share<LAMBDA>, xs: &[&[u8; N]], ys: &mut [&mut [u8; LAMBDA]]) {
        // the crate zips xs with ys (lib.rs:196-198): min(len) points, extra ys rows untouched
        let m = xs.len().min(ys.len());
        self.try_eval(b, k, &xs[..m], &mut ys[..m]).unwrap_or_else(|e| panic!("dcf_eval: {e:?}"))
    }
}

impl<const N: usize, const LAMBDA: usize> Drop for DcfHip<N, LAMBDA> {
    fn drop(&mut self) {
        unsafe { ffi::dcf_prg_free(self.prg) }
    }
}

/// One `Dcf` over several GPUs: `eval` splits the points into contiguous slices (one per
/// device, `dcf_point_slice`) and runs them concurrently (`dcf_eval_multi_gpu`); `gen`
/// runs on the first device.
pub struct DcfHipMulti<const N: usize, const LAMBDA: usize> {
    devs: Vec<DcfHip<N, LAMBDA>>,
}

impl<const N: usize, const LAMBDA: usize> DcfHipMulti<N, LAMBDA> {
    pub fn new(keys: &[&[u8; 32]], devices: &[i32]) -> Result<Self, DcfHipError> {
        let devs = devices.iter().map(|&d| DcfHip::try_new(keys, d)).collect::<Result<Vec<_>, _>>()?;
        Ok(Self { devs })
    }
}

impl<const N: usize, const LAMBDA: usize> Dcf<N, LAMBDA> for DcfHipMulti<N, LAMBDA> {
    fn gen(&self, f: &CmpFn<N, LAMBDA>, s0s: [&[u8; LAMBDA]; 2], bound: BoundState) -> Share<LAMBDA> {
        self.devs[0].gen(f, s0s, bound)
    }

    fn eval(&self, b: bool, k: &Share<LAMBDA>, xs: &[&[u8; N]], ys: &mut [&mut [u8; LAMBDA]]) {
        // the crate zips xs with ys (lib.rs:196-198): min(len) points, extra ys rows untouched
        let m = xs.len().min(ys.len());
        let (xs, ys) = (&xs[..m], &mut ys[..m]);
        let cwb = share_to_cwb::<N, LAMBDA>(k);
        let prgs: Vec<*mut ffi::DcfPrg> = self.devs.iter().map(|d| d.raw()).collect();
        let xb: Vec<u8> = xs.iter().flat_map(|x| x.iter().copied()).collect();
        let mut yb = vec![0u8; ys.len() * LAMBDA];
        check(unsafe {
            ffi::dcf_eval_multi_gpu(prgs.as_ptr(), prgs.len(), N, b as c_int, cwb.as_ptr(), cwb.len(),
                                    k.s0s[0].as_ptr(), xb.as_ptr(), xs.len(), yb.as_mut_ptr(), yb.len())
        })
        .unwrap_or_else(|e| panic!("dcf_eval_multi_gpu: {e:?}"));
        for (y, c) in ys.iter_mut().zip(yb.chunks_exact(LAMBDA)) {
            y.copy_from_slice(c);
        }
    }
}
