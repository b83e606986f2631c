//! The crate's own tests (lib.rs:372-442 of xymeng16/dcf) against DcfHip: same constants,
//! same reconstruction assertions, plus a bit-exact comparison with the crate's CPU
//! DcfImpl on random points (the oracle this backend replaces).  Needs an MI355X.
use dcf::prg::Aes256HirosePrg;
use dcf::{BoundState, CmpFn, Dcf, DcfImpl, Share};
use dcf_hip::{DcfHip, DcfHipMulti};
use rand::{thread_rng, Rng};

const KEYS: [&[u8; 32]; 2] = [
    b"j9\x1b_\xb3X\xf33\xacW\x15\x1b\x0812K\xb3I\xb9\x90r\x1cN\xb5\xee9W\xd3\xbb@\xc6d",
    b"\x9b\x15\xc8\x0f\xb7\xbc!q\x9e\x89\xb8\xf7\x0e\xa0S\x9dN\xfa\x0c;\x16\xe4\x98\x82b\xfcdy\xb5\x8c{\xc2",
];
const ALPHAS: &[&[u8; 16]] = &[
    b"K\xa9W\xf5\xdd\x05\xe9\xfc?\x04\xf6\xfbUo\xa8C",
    b"\xc2GK\xda\xc6\xbb\x99\x98Fq\"f\xb7\x8csU",
    b"\xc2GK\xda\xc6\xbb\x99\x98Fq\"f\xb7\x8csV",
    b"\xc2GK\xda\xc6\xbb\x99\x98Fq\"f\xb7\x8csW",
    b"\xef\x96\x97\xd7\x8f\x8a\xa4AP\n\xb35\xb5k\xff\x97",
];
const BETA: &[u8; 16] = b"\x03\x11\x97\x12C\x8a\xe9#\x81\xa8\xde\xa8\x8f \xc0\xbb";

fn reconstruct(dcf: &impl Dcf<16, 16>, bound: BoundState) -> Vec<[u8; 16]> {
    let s0s: [[u8; 16]; 2] = thread_rng().gen();
    let f = CmpFn { alpha: ALPHAS[2].to_owned(), beta: BETA.to_owned() };
    let k = dcf.gen(&f, [&s0s[0], &s0s[1]], bound);
    let mut k0 = k.clone();
    k0.s0s = vec![k0.s0s[0]];
    let mut k1 = k.clone();
    k1.s0s = vec![k1.s0s[1]];
    let mut ys0 = vec![[0; 16]; ALPHAS.len()];
    let mut ys1 = vec![[0; 16]; ALPHAS.len()];
    dcf.eval(false, &k0, ALPHAS, &mut ys0.iter_mut().collect::<Vec<_>>());
    dcf.eval(true, &k1, ALPHAS, &mut ys1.iter_mut().collect::<Vec<_>>());
    ys0.iter().zip(ys1.iter()).map(|(a, b)| std::array::from_fn(|i| a[i] ^ b[i])).collect()
}

#[test]
fn test_dcf_gen_then_eval_ok() {
    let ys = reconstruct(&DcfHip::<16, 16>::new(KEYS, 0), BoundState::LtBeta);
    assert_eq!(ys, vec![BETA.to_owned(), BETA.to_owned(), [0; 16], [0; 16], [0; 16]]);
}

#[test]
fn test_dcf_gen_gt_beta_then_eval_ok() {
    let ys = reconstruct(&DcfHip::<16, 16>::new(KEYS, 0), BoundState::GtBeta);
    assert_eq!(ys, vec![[0; 16], [0; 16], [0; 16], BETA.to_owned(), BETA.to_owned()]);
}

#[test]
fn test_dcf_gen_then_eval_not_zeros() {
    let dcf = DcfHip::<16, 16>::new(KEYS, 0);
    let s0s: [[u8; 16]; 2] = thread_rng().gen();
    let f = CmpFn { alpha: ALPHAS[2].to_owned(), beta: BETA.to_owned() };
    let k = dcf.gen(&f, [&s0s[0], &s0s[1]], BoundState::LtBeta);
    let mut k0 = k.clone();
    k0.s0s = vec![k0.s0s[0]];
    let mut ys0 = vec![[0; 16]; ALPHAS.len()];
    dcf.eval(false, &k0, ALPHAS, &mut ys0.iter_mut().collect::<Vec<_>>());
    assert_ne!(ys0[2], [0; 16]);
}

#[test]
fn test_bit_exact_with_the_crate_cpu_impl() {
    let cpu = DcfImpl::<16, 16, _>::new(Aes256HirosePrg::<16, 2>::new(KEYS));
    let gpu = DcfHip::<16, 16>::new(KEYS, 0);
    let s0s: [[u8; 16]; 2] = thread_rng().gen();
    let f = CmpFn { alpha: thread_rng().gen(), beta: thread_rng().gen() };
    let k = cpu.gen(&f, [&s0s[0], &s0s[1]], BoundState::LtBeta);
    let kg = gpu.gen(&f, [&s0s[0], &s0s[1]], BoundState::LtBeta);
    assert_eq!(k.cw_np1, kg.cw_np1);
    let xs: Vec<[u8; 16]> = (0..100_000).map(|_| thread_rng().gen()).collect();
    let xr: Vec<&[u8; 16]> = xs.iter().collect();
    for b in [false, true] {
        let kb = Share { s0s: vec![k.s0s[b as usize]], cws: k.cws.clone(), cw_np1: k.cw_np1 };
        let mut yc = vec![[0; 16]; xs.len()];
        let mut yg = vec![[0; 16]; xs.len()];
        cpu.eval(b, &kb, &xr, &mut yc.iter_mut().collect::<Vec<_>>());
        gpu.eval(b, &kb, &xr, &mut yg.iter_mut().collect::<Vec<_>>());
        assert_eq!(yc, yg);
        let multi = DcfHipMulti::<16, 16>::new(&KEYS, &[0]).unwrap();
        let mut ym = vec![[0; 16]; xs.len()];
        multi.eval(b, &kb, &xr, &mut ym.iter_mut().collect::<Vec<_>>());
        assert_eq!(yc, ym);
    }
}

/// `DcfImpl` is `Sync` with a `Sync` PRG (lib.rs:34,52): callers share one instance across
/// threads.  One `DcfHip` driven from 8 threads at once, each with its own key and points,
/// must match the crate's CPU `DcfImpl` bit for bit; and a `ys` longer than `xs` is zipped
/// (lib.rs:196-198): the extra rows stay untouched.
#[test]
fn test_one_instance_many_threads_and_zip_semantics() {
    use std::sync::Arc;
    let cpu = Arc::new(DcfImpl::<16, 16, _>::new(Aes256HirosePrg::<16, 2>::new(KEYS)));
    let gpu = Arc::new(DcfHip::<16, 16>::new(KEYS, 0));
    let handles: Vec<_> = (0..8)
        .map(|i| {
            let (cpu, gpu) = (Arc::clone(&cpu), Arc::clone(&gpu));
            std::thread::spawn(move || {
                let s0s: [[u8; 16]; 2] = thread_rng().gen();
                let f = CmpFn { alpha: thread_rng().gen(), beta: thread_rng().gen() };
                let k = gpu.gen(&f, [&s0s[0], &s0s[1]], BoundState::LtBeta);
                let xs: Vec<[u8; 16]> = (0..[1, 7, 5000, 300_000][i % 4]).map(|_| thread_rng().gen()).collect();
                let xr: Vec<&[u8; 16]> = xs.iter().collect();
                let kb = Share { s0s: vec![k.s0s[0]], cws: k.cws.clone(), cw_np1: k.cw_np1 };
                let mut yc = vec![[0; 16]; xs.len()];
                let mut yg = vec![[0; 16]; xs.len()];
                cpu.eval(false, &kb, &xr, &mut yc.iter_mut().collect::<Vec<_>>());
                gpu.eval(false, &kb, &xr, &mut yg.iter_mut().collect::<Vec<_>>());
                assert_eq!(yc, yg);
            })
        })
        .collect();
    for h in handles {
        h.join().unwrap();
    }
    let s0s: [[u8; 16]; 2] = thread_rng().gen();
    let f = CmpFn { alpha: thread_rng().gen(), beta: thread_rng().gen() };
    let k = gpu.gen(&f, [&s0s[0], &s0s[1]], BoundState::GtBeta);
    let kb = Share { s0s: vec![k.s0s[0]], cws: k.cws.clone(), cw_np1: k.cw_np1 };
    let mut ys = vec![[0xAB; 16]; ALPHAS.len() + 2];
    gpu.eval(false, &kb, ALPHAS, &mut ys.iter_mut().collect::<Vec<_>>());
    assert_eq!(&ys[ALPHAS.len()..], &[[0xAB; 16]; 2]);
}
