// Link libgalahgpu.so (built by `make -C galah_amd/csrc`, hipcc --offload-arch=gfx950).
// GALAHGPU_LIB_DIR overrides the directory; the default is this repository's
// galah_amd/lib next to the crate.  (A link argument of a dependency's build
// script does not reach the final binary: galah's binary finds the library
// through LD_LIBRARY_PATH, or RUSTFLAGS="-C link-arg=-Wl,-rpath,<dir>".)
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = match env::var("GALAHGPU_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../galah_amd/lib"),
    };
    let dir = dir.canonicalize().unwrap_or(dir);
    println!("cargo:rerun-if-env-changed=GALAHGPU_LIB_DIR");
    println!("cargo:rerun-if-changed={}", dir.join("libgalahgpu.so").display());
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=galahgpu");
}
