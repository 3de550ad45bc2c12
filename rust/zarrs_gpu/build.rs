//! Link libzgpu.so (built by `make -C zarrs_amd/csrc` for gfx950). ZGPU_LIB_DIR overrides the location.
fn main() {
    let dir = std::env::var("ZGPU_LIB_DIR").unwrap_or_else(|_| {
        let here = std::env::var("CARGO_MANIFEST_DIR").unwrap_or_else(|_| ".".into());
        format!("{here}/../../zarrs_amd/lib")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=zgpu");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=ZGPU_LIB_DIR");
}
