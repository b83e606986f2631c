//! Raw bindings of include/dcf_hip.h (every entry point; same order as the header).
//! tests/test_rust_ffi.py (in the repo's Python suite) checks names and arities against
//! the header, since this container has no Rust toolchain.
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)]
pub struct DcfPrg {
    _p: [u8; 0],
}

pub const DCF_OK: c_int = 0;
pub const DCF_ERR_ARG: c_int = -1;
pub const DCF_ERR_LAMBDA: c_int = -2;
pub const DCF_ERR_CIPHER_N: c_int = -3;
pub const DCF_ERR_N: c_int = -4;
pub const DCF_ERR_LEN: c_int = -5;
pub const DCF_ERR_HIP: c_int = -6;
pub const DCF_ERR_UNSUPPORTED: c_int = -7;
pub const DCF_ERR_KEY: c_int = -8;

extern "C" {
    pub fn dcf_version() -> *const c_char;
    pub fn dcf_last_error() -> *const c_char;
    pub fn dcf_hirose_prg_new(keys: *const u8, cipher_n: usize, lambda: usize, device: c_int,
                              out: *mut *mut DcfPrg) -> c_int;
    pub fn dcf_mmo_prg_new(keys: *const u8, cipher_n: usize, lambda: usize, device: c_int,
                           out: *mut *mut DcfPrg) -> c_int;
    pub fn dcf_prg_kind(prg: *const DcfPrg) -> c_int;
    pub fn dcf_prg_free(prg: *mut DcfPrg);
    pub fn dcf_prg_lambda(prg: *const DcfPrg) -> usize;
    pub fn dcf_prg_set_eval_mode(prg: *mut DcfPrg, mode: c_int) -> c_int;
    pub fn dcf_prg_set_prefix_levels(prg: *mut DcfPrg, levels: c_int) -> c_int;
    pub fn dcf_eval_prefix_levels(prg: *const DcfPrg, n_bytes: usize, num_keys: usize, points_per_key: usize) -> c_int;
    pub fn dcf_eval_keys_per_launch(n_bytes: usize, points_per_key: usize) -> usize;
    pub fn dcf_prg_set_prefix_max_bytes(prg: *mut DcfPrg, max_bytes: usize) -> c_int;
    pub fn dcf_prg_device_bytes(prg: *const DcfPrg) -> usize;
    pub fn dcf_prg_host_pinned_bytes(prg: *const DcfPrg) -> usize;
    pub fn dcf_prg_workspaces(prg: *const DcfPrg) -> c_int;
    pub fn dcf_prg_trim(prg: *mut DcfPrg) -> c_int;
    pub fn dcf_prg_last_eval_blocks(prg: *mut DcfPrg, blocks: *mut u64) -> c_int;
    pub fn dcf_prg_set_phase_timing(prg: *mut DcfPrg, on: c_int) -> c_int;
    pub fn dcf_prg_last_eval_phases(prg: *mut DcfPrg, prep_ms: *mut f32, walk_ms: *mut f32,
                                    prefix_levels: *mut c_int) -> c_int;
    pub fn dcf_cwb_bytes(n_bytes: usize, lambda: usize, num_keys: usize) -> usize;
    pub fn dcf_cwb_np1_offset(n_bytes: usize, lambda: usize, num_keys: usize) -> usize;
    pub fn dcf_gen(prg: *mut DcfPrg, n_bytes: usize, alpha: *const u8, beta: *const u8, s0_0: *const u8,
                   s0_1: *const u8, bound: c_int, cwb_out: *mut u8) -> c_int;
    pub fn dcf_eval(prg: *mut DcfPrg, n_bytes: usize, party: c_int, cwb: *const u8, cwb_len: usize, s0: *const u8,
                    xs: *const u8, m: usize, ys: *mut u8, ys_len: usize) -> c_int;
    pub fn dcf_prg_gen(prg: *mut DcfPrg, seeds: *const u8, m: usize, out: *mut u8) -> c_int;
    pub fn dcf_gen_batch_device(prg: *mut DcfPrg, n_bytes: usize, num_keys: usize, alpha: *const u8,
                                beta: *const u8, s0_0: *const u8, s0_1: *const u8, bound: c_int,
                                cwb_out: *mut u8, stream: *mut c_void) -> c_int;
    pub fn dcf_eval_device(prg: *mut DcfPrg, n_bytes: usize, party: c_int, cwb: *const u8, s0: *const u8,
                           xs: *const u8, m: usize, ys: *mut u8, stream: *mut c_void) -> c_int;
    pub fn dcf_eval_multikey_device(prg: *mut DcfPrg, n_bytes: usize, num_keys: usize, points_per_key: usize,
                                    party: c_int, cwb: *const u8, s0s: *const u8, xs: *const u8, ys: *mut u8,
                                    stream: *mut c_void) -> c_int;
    pub fn dcf_point_slice(total: usize, g_count: usize, g: usize, start: *mut usize, count: *mut usize);
    pub fn dcf_eval_multi_gpu(prgs: *const *mut DcfPrg, g_count: usize, n_bytes: usize, party: c_int,
                              cwb: *const u8, cwb_len: usize, s0: *const u8, xs: *const u8, m: usize,
                              ys: *mut u8, ys_len: usize) -> c_int;
    pub fn dcf_eval_multi_gpu_device(prgs: *const *mut DcfPrg, g_count: usize, n_bytes: usize, party: c_int,
                                     cwb: *const u8, cwb_len: usize, s0: *const u8, xs: *const *const u8,
                                     ms: *const usize, ys: *const *mut u8, streams: *const *mut c_void,
                                     gather_ys: *mut u8) -> c_int;
    pub fn dcf_share_bincode_bytes(n_bytes: usize, lambda: usize, num_s0s: usize) -> usize;
    pub fn dcf_share_to_bincode(n_bytes: usize, lambda: usize, cwb: *const u8, s0s: *const u8, num_s0s: usize,
                                out: *mut u8, out_len: usize) -> c_int;
    pub fn dcf_share_from_bincode(n_bytes: usize, lambda: usize, inp: *const u8, in_len: usize, cwb_out: *mut u8,
                                  s0s_out: *mut u8, max_s0s: usize, num_s0s: *mut usize) -> c_int;
    pub fn dcf_eval_full_domain_device(prg: *mut DcfPrg, n_bytes: usize, party: c_int, cwb: *const u8,
                                       s0: *const u8, ys: *mut u8, stream: *mut c_void) -> c_int;
}
