//! Generates the bindings of include/capsule_gpu.h and links libcapsule_gpu.so
//! and the HIP runtime, the way the reference's ffi/build.rs:171-216 binds
//! DPDK (allow-list by prefix, derive_default, rerun-if-changed).
//!
//! CAPSULE_GPU_ROOT: a checkout of this repository with the library built
//! (`make -C capsule_amd/csrc`, i.e. capsule_amd/libcapsule_gpu.so).
//! ROCM_PATH: the ROCm install (default /opt/rocm), for libamdhip64.
use std::env;
use std::path::PathBuf;

fn main() {
    let root = PathBuf::from(env::var("CAPSULE_GPU_ROOT").expect("CAPSULE_GPU_ROOT: the capsule_amd checkout"));
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".to_string());
    let header = root.join("include").join("capsule_gpu.h");

    bindgen::Builder::default()
        .header(header.to_str().expect("utf-8 path"))
        .whitelist_type(r"cgpu_.*")
        .whitelist_function(r"cgpu_.*")
        .whitelist_var(r"CGPU_.*")
        .derive_copy(true)
        .derive_debug(true)
        .derive_default(true)
        .default_enum_style(bindgen::EnumVariation::ModuleConsts)
        .rustfmt_bindings(true)
        .generate()
        .expect("Unable to generate capsule_gpu bindings")
        .write_to_file(PathBuf::from(env::var("OUT_DIR").unwrap()).join("bindings.rs"))
        .expect("Couldn't write bindings!");

    println!("cargo:rustc-link-search=native={}", root.join("capsule_amd").display());
    println!("cargo:rustc-link-lib=dylib=capsule_gpu");
    println!("cargo:rustc-link-search=native={}/lib", rocm);
    println!("cargo:rustc-link-lib=dylib=amdhip64");
    println!("cargo:rerun-if-changed=build.rs");
    println!("cargo:rerun-if-changed={}", header.display());
    println!("cargo:rerun-if-env-changed=CAPSULE_GPU_ROOT");
}
