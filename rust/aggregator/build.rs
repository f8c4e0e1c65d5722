// aggregator/build.rs -- the reference's script (records the rustc version for
// `env!("RUSTC_SEMVER")`, aggregator/src/metrics.rs:227) plus, with the `mi355x` feature, the
// build of the MI355X engine (this repository) with hipcc.
// Not compiled here (no cargo in this image); mirrors janus_amd/_lib.py::build(), including the
// build hash the library embeds (prio3gpu_build_hash) so gpu::check_build can reject a stale one.
use rustc_version::version;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    // the reference's build script, unchanged (aggregator/build.rs:3-6)
    let rustc_semver = version().expect("could not parse rustc version");
    println!("cargo:rustc-env=RUSTC_SEMVER={rustc_semver}");
    println!("cargo:rerun-if-env-changed=RUSTC");

    if std::env::var("CARGO_FEATURE_MI355X").is_err() {
        return;
    }
    println!("cargo:rerun-if-env-changed=PRIO3GPU_ROOT");
    let root = PathBuf::from(std::env::var("PRIO3GPU_ROOT").unwrap_or("../prio3-mi355x".into()));
    let csrc = root.join("janus_amd/csrc");
    let out = PathBuf::from(std::env::var("OUT_DIR").unwrap());
    // the same key janus_amd/_lib.py::source_hash computes (sources, headers, flags); a failed
    // python3 (missing, wrong PRIO3GPU_ROOT) must stop the build, never yield an empty hash that
    // would disable gpu::check_build
    let py = Command::new("python3")
        .args(["-c", "from janus_amd import _lib; print(_lib.source_hash(), end='')"])
        .current_dir(&root)
        .output()
        .expect("python3 not found: needed to compute the engine's build hash");
    assert!(
        py.status.success(),
        "computing the engine build hash failed (PRIO3GPU_ROOT={}): {}",
        root.display(),
        String::from_utf8_lossy(&py.stderr)
    );
    let hash = String::from_utf8(py.stdout).expect("build hash is not UTF-8");
    assert!(
        hash.len() == 64 && hash.bytes().all(|b| b.is_ascii_hexdigit()),
        "bad engine build hash {hash:?}"
    );
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
