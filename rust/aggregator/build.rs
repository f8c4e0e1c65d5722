// aggregator/build.rs -- the reference's script records the rustc version; with the `mi355x`
// feature it also builds the MI355X engine (this repository) with hipcc and links it.
// Not compiled here (no cargo in this image); mirrors janus_amd/_lib.py::build(), including the
// build hash the library embeds (prio3gpu_build_hash) so gpu::check_build can reject a stale one.
use std::path::PathBuf;
use std::process::Command;

fn main() {
    // (the reference's rustc-version recording stays as it is)
    if std::env::var("CARGO_FEATURE_MI355X").is_err() {
        return;
    }
    let root = PathBuf::from(std::env::var("PRIO3GPU_ROOT").unwrap_or("../prio3-mi355x".into()));
    let csrc = root.join("janus_amd/csrc");
    let out = PathBuf::from(std::env::var("OUT_DIR").unwrap());
    // the same key janus_amd/_lib.py::source_hash computes (sources, headers, flags)
    let hash = String::from_utf8(
        Command::new("python3")
            .args(["-c", "from janus_amd import _lib; print(_lib.source_hash(), end='')"])
            .current_dir(&root)
            .output()
            .expect("python3")
            .stdout,
    )
    .unwrap();
    let status = Command::new("hipcc")
        .args(["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared"])
        .arg(format!("-DPRIO3GPU_BUILD_HASH=\"{hash}\""))
        .arg("-o")
        .arg(out.join("libprio3gpu.so"))
        .args(["engine.hip", "codec.cpp", "hpke.cpp"].iter().map(|f| csrc.join(f)))
        .args(["-lrccl", "-lcrypto"])
        .status()
        .expect("hipcc");
    assert!(status.success(), "hipcc failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=prio3gpu");
    println!("cargo:rustc-env=PRIO3GPU_BUILD_HASH={hash}");
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", root.join("include/prio3gpu.h").display());
}
