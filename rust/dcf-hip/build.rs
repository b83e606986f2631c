// Links libdcf_hip.so (built by `python -m dcf_amd.build`, hipcc --offload-arch=gfx950).
// DCF_HIP_LIB_DIR: directory holding libdcf_hip.so (default: ../../dcf_amd of this repo).
fn main() {
    let dir = std::env::var("DCF_HIP_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap();
        format!("{here}/../../dcf_amd")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=dcf_hip");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=DCF_HIP_LIB_DIR");
}
