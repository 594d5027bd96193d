"""The product's host Blake2s (r1cs-spartan_amd/csrc/transcript.hpp, the Fiat-Shamir transcript's
hash): RFC 7693 known answer and piecewise-update consistency, compiled from the header on the host
(no GPU). Its use inside the transcript is pinned by every FS proof of the GPU parity tests."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_blake2s_kat_and_pieces(tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "b2check")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-w", "-I", os.path.join(ROOT, "r1cs-spartan_amd", "csrc"),
                           "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                           os.path.join(ROOT, "tests", "native", "blake2s_check.cpp"), "-o", exe])
    out = subprocess.check_output([exe], timeout=120).decode()
    assert out.startswith("ok"), out


def test_sumcheck1_message_stepping(tmp_path):
    """prover.cpp's sumcheck-1 message (finite differences, sc_message.hpp) equals the point-by-point
    Lagrange form of P(t) = C eq(tau, t) G(t) (prover.rs:199-207 with the degree-3 factorisation)"""
    cxx = shutil.which("g++") or shutil.which("clang++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "scmsg")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-w", "-I", os.path.join(ROOT, "r1cs-spartan_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "sc_message_check.cpp"), "-o", exe])
    out = subprocess.check_output([exe], timeout=120).decode()
    assert out.startswith("ok"), out


def test_blake2s_lanes_match_scalar(tmp_path):
    """blake2s_lanes.cpp (multi-buffer absorption of several proofs' matrices): every lane equals a
    scalar stream over the same pieces, for lane counts below / at / above the vector width"""
    cxx = shutil.which("g++") or shutil.which("clang++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "b2lanes")
    csrc = os.path.join(ROOT, "r1cs-spartan_amd", "csrc")
    subprocess.check_call([cxx, "-O3", "-std=c++17", "-w", "-I", csrc, os.path.join(csrc, "blake2s_lanes.cpp"),
                           os.path.join(ROOT, "tests", "native", "blake2s_lanes_check.cpp"), "-o", exe])
    out = subprocess.check_output([exe], timeout=300).decode()
    assert out.startswith("ok"), out
    print(out)


def test_hash_pool_schedule(tmp_path):
    """spx_prove_many's hashing-pool plan (csrc/hash_sched.hpp): every owned proof absorbed exactly once
    for any pool size / context count / lane width, the first two waves one proof per job, and every
    pool thread terminates"""
    cxx = shutil.which("g++") or shutil.which("clang++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "hsched")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "r1cs-spartan_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "hash_sched_check.cpp"), "-o", exe])
    out = subprocess.check_output([exe], timeout=300).decode()
    assert out.startswith("ok"), out
