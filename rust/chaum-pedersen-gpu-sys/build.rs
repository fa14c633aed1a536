//! Builds libcpz.so for gfx950 with hipcc (the same recipe as
//! chaum-pedersen-zkp_amd/build_native.py) and links it.  The reference crate's own build.rs
//! (tonic-build under the `grpc` feature, build.rs:1-12) stays unchanged: the HIP step lives
//! here, so only builds that enable the GPU path need ROCm.
//!
//! Environment:
//!   CPZ_LIB_DIR      use a prebuilt libcpz.so from this directory instead of compiling
//!   CPZ_SRC_DIR      the csrc/ directory (default: ../../chaum-pedersen-zkp_amd/csrc)
//!   CPZ_OFFLOAD_ARCH offload target (default gfx950)
//!   HIPCC            the hipcc binary (default: $ROCM_PATH/bin/hipcc or /opt/rocm/bin/hipcc)
use std::env;
use std::path::PathBuf;
use std::process::Command;

const UNITS: [&str; 5] = ["kernels.hip", "wide.hip", "rlc.hip", "part.hip", "runtime.hip"];

fn main() {
    println!("cargo:rerun-if-env-changed=CPZ_LIB_DIR");
    println!("cargo:rerun-if-env-changed=CPZ_SRC_DIR");
    println!("cargo:rerun-if-env-changed=CPZ_OFFLOAD_ARCH");
    if let Ok(dir) = env::var("CPZ_LIB_DIR") {
        println!("cargo:rustc-link-search=native={dir}");
        println!("cargo:rustc-link-lib=dylib=cpz");
        return;
    }
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let src = env::var("CPZ_SRC_DIR")
        .map(PathBuf::from)
        .unwrap_or_else(|_| manifest.join("../../chaum-pedersen-zkp_amd/csrc"));
    let include = src.join("../../include");
    let arch = env::var("CPZ_OFFLOAD_ARCH").unwrap_or_else(|_| "gfx950".into());
    let rocm = env::var("ROCM_PATH").unwrap_or_else(|_| "/opt/rocm".into());
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| format!("{rocm}/bin/hipcc"));
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    let mut objs = Vec::new();
    for unit in UNITS {
        let input = src.join(unit);
        println!("cargo:rerun-if-changed={}", input.display());
        let obj = out.join(unit.replace(".hip", ".o"));
        // build_native.py's UNIT_FLAGS: aligned loop heads for the row kernels
        let unit_flags: &[&str] = if unit == "wide.hip" { &["-falign-loops=64"] } else { &[] };
        let st = Command::new(&hipcc)
            .args([&format!("--offload-arch={arch}"), "-O3", "-std=c++17", "-fPIC", "-c"])
            .args(unit_flags)
            .arg("-I").arg(&src)
            .arg("-I").arg(&include)
            .arg(&input).arg("-o").arg(&obj)
            .status()
            .expect("hipcc not found: set HIPCC / ROCM_PATH, or CPZ_LIB_DIR to a prebuilt libcpz.so");
        assert!(st.success(), "hipcc failed on {}", input.display());
        objs.push(obj);
    }
    for h in std::fs::read_dir(&src).unwrap().flatten() {
        if h.path().extension().map_or(false, |e| e == "h") {
            println!("cargo:rerun-if-changed={}", h.path().display());
        }
    }
    println!("cargo:rerun-if-changed={}", include.join("cpz.h").display());
    let lib = out.join("libcpz.so");
    let st = Command::new(&hipcc)
        .args([&format!("--offload-arch={arch}"), "-shared", "-fPIC", "-o"])
        .arg(&lib)
        .args(&objs)
        .status()
        .expect("hipcc link step");
    assert!(st.success(), "hipcc link failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=cpz");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
}
