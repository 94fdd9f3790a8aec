"""The C-ABI boundary on the CPU: the library loads, exports every symbol include/bcfft.h
declares, and validates arguments before launching anything (no GPU needed for that)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bcfft.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bcfft_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ("bcfft_forward", "bcfft_spectra", "bcfft_spectra_bytes", "bcfft_circulant_matvec",
              "bcfft_abi_version", "bcfft_status_string", "bcfft_last_hip_error"):
        assert f in fns


def test_library_exports_every_header_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    for f in header_functions():
        assert hasattr(lib, f), f"{f} declared in bcfft.h but not exported"


def test_binding_signatures_cover_header(built_lib):
    from bcfft import _lib
    assert set(_lib._SIGNATURES) == set(header_functions())
    lib = _lib.load()
    assert lib.bcfft_abi_version() == _lib.ABI_VERSION


def test_status_strings_and_sizes(built_lib):
    from bcfft import _lib
    lib = _lib.load()
    assert lib.bcfft_status_string(0) == b"ok"
    assert b"block_size" in lib.bcfft_status_string(2)
    # (nO*nI*b/2 + b) complex64 + split-bf16 MFMA image (b <= 128):
    # ceil(nI/8) chunks x b/2 bins x {hi,lo} x nO padded to 4096/b x 8 blocks x 4 B
    # + stationary image where eligible: 16-B header + ceil(nO/32) groups x 8 waves x
    #   (b/16 bins x nI/16 K-steps x 2 N-tiles) x 64 lanes x 16 B
    # + streamed image for b = 128, nI > 32 (bcfft_dmk.hip): 16-B header + ceil(nO/32) groups x
    #   ceil(nI/16) chunks x (8 waves x 8 bins x 2 N-tiles) x 64 lanes x 16 B
    def expect(no, ni, b):
        img = 0
        if b <= 128:
            opw = 4096 // b
            img = -(-ni // 8) * (b // 2) * 2 * (-(-no // opw) * opw) * 8 * 4
        # (+ the per-output-block inverse weight scales: 32 fp32 per group)
        stat = 0
        if (b == 128 and ni == 32) or (b == 64 and (ni in (32, 64) or 64 < ni <= 255)) or (b == 256 and 1 <= ni <= 127):
            stat = 16 + -(-no // 32) * 8 * ((b // 16) * -(-ni // 16) * 2) * 64 * 16 + -(-no // 32) * 32 * 4
        elif b == 128 and 32 < ni <= 127:
            stat = 16 + -(-no // 32) * -(-ni // 16) * 128 * 64 * 16 + -(-no // 32) * 32 * 4
        # + the precise engine's e4m3 weight residual (b = 128, K = 4096): per group 8 waves x 8 bins x
        #   2 K-steps x 64 lanes x 16 B
        lo8 = -(-no // 32) * 8 * 8 * 2 * 64 * 16 if (b == 128 and ni == 32) else 0
        return (no * ni * (b // 2) + b) * 8 + img + stat + lo8
    for no, ni, b in [(32, 32, 128), (86, 32, 128), (32, 86, 128), (40, 48, 128), (8, 160, 128), (64, 64, 64), (2, 4, 32), (16, 16, 256), (16, 43, 256), (43, 8, 256), (2, 128, 256), (64, 172, 64), (3, 256, 64)]:
        assert lib.bcfft_spectra_bytes(no, ni, b) == expect(no, ni, b)
    assert lib.bcfft_spectra_bytes(2, 2, 100) == -1
    assert lib.bcfft_spectra_bytes(0, 2, 64) == -1


def test_argument_validation_without_launch(built_lib):
    """Every rejected call returns before any HIP launch, so this runs without a GPU."""
    from bcfft import _lib
    lib = _lib.load()
    F32, BF16, NONE = _lib.BCFFT_F32, _lib.BCFFT_BF16, _lib.BCFFT_NONE
    fake = 4096  # never dereferenced: validation fails first
    fwd = lib.bcfft_forward
    assert fwd(fake, F32, 8, 4096, 4096, 100, fake, None, NONE, fake, F32, None) == 2   # block
    assert fwd(fake, F32, 8, 4000, 4096, 128, fake, None, NONE, fake, F32, None) == 1   # shape
    assert fwd(fake, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, BF16, None) == 3  # y dtype
    assert fwd(fake, BF16, 8, 4096, 4096, 128, fake, fake, F32, fake, BF16, None) == 3  # promote
    assert fwd(fake, 7, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, None) == 3     # dtype
    assert fwd(fake, F32, 8, 4096, 4096, 128, fake, fake, NONE, fake, F32, None) == 6   # bias arg
    assert fwd(None, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, None) == 6   # NULL x
    assert fwd(fake + 4, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, None) == 4  # align
    assert fwd(None, F32, 0, 4096, 4096, 128, None, None, NONE, None, F32, None) == 0   # N=0 no-op
    fa = lib.bcfft_forward_algo
    assert fa(fake, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, 9, None) == 6   # bad algo
    assert fa(None, F32, 0, 4096, 4096, 128, None, None, NONE, None, F32, 2, None) == 0
    glu = lib.bcfft_forward_glu_algo
    assert glu(fake, F32, 8, 4096, 11008, 256, fake, fake, 0, None) == 2      # b = 256 GLU: bf16 only
    assert glu(fake, BF16, 8, 4096, 11008, 256, fake, fake, 3, None) == 2     # ... and no stationary form
    spec = lib.bcfft_spectra
    assert spec(fake, F32, 2, 2, 48, 0, fake, None) == 2
    assert spec(None, F32, 2, 2, 64, 0, fake, None) == 6
    assert spec(fake, F32, 0, 2, 64, 0, fake, None) == 1
    assert spec(fake, F32, 2, 2, 64, 0, fake + 8, None) == 4
    assert lib.bcfft_circulant_matvec(fake, fake, F32, 0, fake, None) == 1


def test_python_layer_fails_loudly_on_cpu_tensors(built_lib):
    import torch
    from bcfft import ops
    with pytest.raises(RuntimeError, match="ROCm device"):
        ops.forward(torch.zeros(2, 128), torch.zeros(10), None, 64, 128)
    with pytest.raises(RuntimeError, match="ROCm device"):
        ops.spectra(torch.zeros(2, 2, 64))


def _device_disassembly(lib_path, tmp_path):
    import subprocess
    llvm = "/opt/rocm/lib/llvm/bin"
    fat = os.path.join(tmp_path, "fat.bin")
    dev = os.path.join(tmp_path, "dev.o")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib_path, fat], check=True)
    subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True)
    return subprocess.run([f"{llvm}/llvm-objdump", "-d", dev], check=True, capture_output=True,
                          text=True).stdout


def test_gfx950_code_object_has_no_packed_fp32(built_lib, tmp_path):
    """Regression guard (DESIGN.md, gfx950 packed-FP32 hazard): packed-FP32 VALU ops running
    beside another wave's MFMAs on the same SIMD corrupted lanes 48-63; the build disables SLP
    vectorisation so no v_pk_{add,mul,fma}_f32 may appear. Also checks the MFMA path exists."""
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("ROCm llvm tools not present")
    asm = _device_disassembly(built_lib, str(tmp_path))
    assert re.search(r"v_pk_(add|mul|fma)_f32", asm) is None
    assert "v_mfma_f32_16x16x32_bf16" in asm
    assert "global_load_lds_dword" in asm


def test_forward_workspace_bytes_without_gpu(built_lib):
    """Split-K workspace sizing is host logic: non-zero only where the MFMA kernel runs a grid of
    fewer 8-token rows than CUs over >= 4 chunks of 8 input blocks (no GPU here: 256 CUs)."""
    from bcfft import _lib
    lib = _lib.load()
    ws = lib.bcfft_forward_workspace_bytes
    AUTO, MFMA, VALU, STAT = (_lib.ALGOS[a] for a in ("auto", "mfma", "valu", "stationary"))
    assert ws(100, 11008, 4096, 128, AUTO) == 6 * 100 * 4096 * 4       # 13 rows: 6 slices of 2 chunks
    assert ws(20, 11008, 4096, 128, AUTO) == 11 * 20 * 4096 * 4        # decode batch: 1 chunk per slice
    assert ws(40, 11008, 4096, 128, AUTO) == 6 * 40 * 4096 * 4         # 5 rows: 2 chunks per slice
    assert ws(1024, 11008, 4096, 128, AUTO) == 4 * 1024 * 4096 * 4     # 128 rows: 4 slices (3,3,3,2)
    assert ws(1700, 11008, 4096, 128, AUTO) == 2 * 1700 * 4096 * 4     # prefill batch: 2 slices
    assert ws(2040, 11008, 4096, 128, AUTO) == 2 * 2040 * 4096 * 4     # 255 rows < 256 CUs
    assert ws(2048, 11008, 4096, 128, AUTO) == 0                    # 256 rows: full grid
    assert ws(100, 4096, 4096, 128, AUTO) == 0                      # DFT kernel (persistent)
    assert ws(100, 4096, 4096, 128, MFMA) == 2 * 100 * 4096 * 4        # forced MFMA: 4 chunks
    assert ws(100, 3072, 4096, 128, MFMA) == 0                      # 3 chunks: never split
    assert ws(50, 11008, 4096, 128, VALU) == 22 * 50 * 4096 * 4     # VALU b = 128: 22 chunks of 4 blocks
    assert ws(20, 4096, 4096, 256, AUTO) == 4 * 20 * 4096 * 4       # VALU b = 256: 4 chunks, 1 per slice
    assert ws(37, 11008, 4096, 256, AUTO) == 11 * 37 * 4096 * 4     # VALU b = 256: 11 chunks
    assert ws(2048, 4096, 4096, 256, AUTO) == 2 * 2048 * 4096 * 4   # 128 rows, 1 workgroup per CU: 2 slices
    assert ws(4096, 4096, 4096, 256, AUTO) == 0                     # 256 rows: full grid
    assert ws(100, 3072, 4096, 256, AUTO) == 0                      # 12 blocks: 3 chunks
    assert ws(100, 4000, 4096, 128, AUTO) == -1
    assert ws(0, 11008, 4096, 128, AUTO) == 0
    fake = 4096
    F32, NONE = _lib.BCFFT_F32, _lib.BCFFT_NONE
    fw = lib.bcfft_forward_ws
    assert fw(fake, F32, 8, 11008, 4096, 128, fake, None, NONE, fake, F32, AUTO, fake + 4, 1 << 20, None) == 4
    assert fw(None, F32, 0, 11008, 4096, 128, None, None, NONE, None, F32, AUTO, None, 0, None) == 0
    assert fw(fake, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, 9, None, 0, None) == 6


def test_forward_workspace_bytes_io_follows_the_engine(built_lib):
    """With the I/O dtypes known, AUTO resolves exactly as the forward will: the bf16 down
    projection (streamed-weight DFT kernel) and b = 64 bf16 (DFT kernel) take no workspace, while
    the same geometries with fp32 I/O still split K on the MFMA kernel."""
    from bcfft import _lib
    lib = _lib.load()
    wio = lib.bcfft_forward_workspace_bytes_io
    AUTO, MFMA = _lib.ALGOS["auto"], _lib.ALGOS["mfma"]
    F32, BF16 = _lib.BCFFT_F32, _lib.BCFFT_BF16
    assert wio(100, 11008, 4096, 128, AUTO, BF16, BF16) == 6 * 100 * 4096 * 4   # dmk K-chunk split: 6 slices
    assert wio(128, 11008, 4096, 128, AUTO, BF16, BF16) == 6 * 128 * 4096 * 4    # 16 tiles: still split
    assert wio(136, 11008, 4096, 128, AUTO, BF16, BF16) == 0                    # 17 tiles: unsplit
    assert wio(100, 11008, 4096, 128, AUTO, F32, F32) == 6 * 100 * 4096 * 4
    assert wio(100, 11008, 4096, 128, AUTO, BF16, F32) == 6 * 100 * 4096 * 4   # fp32 bias: not dmk
    assert wio(100, 11008, 4096, 128, MFMA, BF16, BF16) == 6 * 100 * 4096 * 4  # forced MFMA splits
    assert wio(100, 4096, 11008, 64, AUTO, BF16, BF16) == 0
    assert wio(100, 4096, 4096, 128, AUTO, F32, F32) == 0
    assert wio(100, 4096, 4096, 128, AUTO, 7, F32) == -1


def test_refusal_names_engine_and_geometry(built_lib):
    """BCFFT_ERR_BLOCK comes with the refused engine and geometry (bcfft_last_error_detail),
    before anything is launched."""
    from bcfft import _lib
    lib = _lib.load()
    fake, F32, NONE = 4096, _lib.BCFFT_F32, _lib.BCFFT_NONE
    st = lib.bcfft_forward_ws(fake, F32, 8, 4096, 4096, 64, fake, None, NONE, fake, F32, _lib.ALGOS["dft"],
                              None, 0, None)
    assert st == 2
    d = lib.bcfft_last_error_detail().decode()
    assert "'dft'" in d and "block_size 64" in d and "64 input blocks" in d and "x fp32" in d, d
    with pytest.raises(RuntimeError, match="engine 'dft' does not serve block_size 64"):
        _lib.check(st, "bcfft_forward")
    assert lib.bcfft_forward_ws(None, F32, 0, 4096, 4096, 128, None, None, NONE, None, F32, 0, None, 0, None) == 0
    assert lib.bcfft_last_error_detail().decode() == ""


def test_mlp_mode_and_workspace_without_gpu(built_lib):
    """bcfft_forward_mlp's mode resolution is host logic: the one-launch kernel (no workspace) for
    bf16 at b = 128, hidden 4096, intermediate 33..127 blocks; the split form's workspace is h;
    a forced FUSED on another geometry is refused with its reason before any launch."""
    from bcfft import _lib
    lib = _lib.load()
    wb = lib.bcfft_forward_mlp_workspace_bytes
    AUTO, FUSED, SPLIT = (_lib.MLP_MODES[m] for m in ("auto", "fused", "split"))
    F32, BF16 = _lib.BCFFT_F32, _lib.BCFFT_BF16
    assert wb(8192, 4096, 11008, 128, BF16, AUTO) == 0
    assert wb(768, 4096, 11008, 128, BF16, AUTO) == 2 * 768 * 4096 * 4  # 96 tiles: group split, 2 slices
    assert wb(1100, 4096, 11008, 128, BF16, AUTO) == 0                 # 138 tiles: one launch
    assert wb(760, 4096, 11008, 128, BF16, AUTO) == 2 * 760 * 4096 * 4   # fewer: group split, 2 slices
    assert wb(20, 4096, 11008, 128, BF16, AUTO) == 6 * 20 * 4096 * 4     # decode: 6 slices of 1 group
    FSK = _lib.MLP_MODES["fused_splitk"]
    mm = lib.bcfft_forward_mlp_mode
    assert mm(20, 4096, 11008, 128, BF16, AUTO) == FSK and mm(8192, 4096, 11008, 128, BF16, AUTO) == FUSED
    assert mm(2380, 4096, 11008, 128, BF16, AUTO) == SPLIT and mm(20, 4096, 11008, 128, F32, AUTO) == SPLIT
    assert mm(8192, 4096, 11008, 128, BF16, FSK) == FUSED                # nothing to split: one launch
    assert wb(20, 4096, 11008, 128, BF16, FUSED) == 0 and wb(20, 4096, 11008, 128, BF16, SPLIT) == 20 * 11008 * 2
    assert wb(2380, 4096, 11008, 128, BF16, AUTO) == 2380 * 11008 * 2    # 298 tiles: 2 thin rounds
    assert wb(3072, 4096, 11008, 128, BF16, AUTO) == 0                   # 2 rounds of 192 tiles
    assert wb(1, 4096, 11008, 128, BF16, FUSED) == 0
    assert wb(8192, 4096, 11008, 128, BF16, SPLIT) == 8192 * 11008 * 2
    assert wb(7, 4096, 11008, 128, F32, AUTO) == (7 * 11008 * 4 + 15) // 16 * 16   # fp32: split
    assert wb(5, 4096, 11008, 64, BF16, AUTO) == 5 * 11008 * 2                      # b = 64: split
    assert wb(5, 4096, 4096, 128, BF16, AUTO) == 5 * 4096 * 2                       # 32 h blocks: split
    assert wb(5, 4096, 16384, 128, BF16, AUTO) == 5 * 16384 * 2                     # 128 h blocks: split
    assert wb(2048, 4096, 16256, 128, BF16, AUTO) == 0                              # 127 h blocks
    assert wb(5, 4096, 11008, 128, BF16, 4) == -1
    assert wb(5, 4000, 11008, 128, BF16, AUTO) == -1
    fake = 4096
    fm = lib.bcfft_forward_mlp
    assert fm(fake, F32, 8, 4096, 11008, 128, fake, fake, fake, FUSED, None, 0, None) == 2
    d = lib.bcfft_last_error_detail().decode()
    assert "bcfft_forward_mlp" in d and "x fp32" in d and "intermediate 11008" in d, d
    assert fm(fake, BF16, 8, 4096, 11008, 128, fake, fake, fake, SPLIT, None, 0, None) == 6   # no workspace
    assert fm(fake, BF16, 8, 4096, 11008, 128, fake, fake, fake + 2, FUSED, None, 0, None) == 4   # y misaligned
    assert fm(None, BF16, 0, 4096, 11008, 128, None, None, None, AUTO, None, 0, None) == 0
    assert fm(fake, BF16, 8, 4096, 11008, 128, fake, fake, fake, 7, None, 0, None) == 6
