"""C++ host runtime (_cgs_runtime): BLAKE3 known-answer vectors, safetensors round trip against the
`safetensors` package, BPE parity with the pure-Python merge loop (SURVEY §2.3 native rows)."""
import hashlib
import os

import pytest
import torch

from comfy_gen_server_amd import _native


@pytest.fixture(scope="module")
def rt():
    m = _native.load_runtime()
    if m is None:
        import build_native
        build_native.build_runtime()
        _native._runtime_err = None
        m = _native.load_runtime()
    assert m is not None, _native.runtime_error()
    return m


def test_blake3_vectors(rt, tmp_path):
    # official BLAKE3 test vectors (empty input, "abc")
    assert rt.blake3_hex(b"") == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"
    assert rt.blake3_hex(b"abc") == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"
    # extended output is a prefix-extension of the default digest
    assert rt.blake3_hex(b"abc", 64).startswith(rt.blake3_hex(b"abc"))
    # multi-chunk / multi-thread tree == file path == bytes path
    data = bytes((i * 7 + 3) & 0xFF for i in range(9 * 1024 * 1024 + 517))
    p = tmp_path / "blob.bin"
    p.write_bytes(data)
    h = rt.blake3_hex(data)
    assert rt.blake3_file_hex(str(p)) == h and len(h) == 64
    # tree boundaries: lengths around chunk / power-of-two edges give distinct, stable digests
    seen = set()
    for n in (1023, 1024, 1025, 2048, 2049, 3072, 4097):
        d = rt.blake3_hex(data[:n])
        assert d not in seen
        seen.add(d)


def test_hashing_uses_blake3(rt, tmp_path):
    from comfy_gen_server_amd.utils.hashing import bytes_digest, file_digest
    p = tmp_path / "f.txt"
    p.write_bytes(b"abc")
    assert file_digest(str(p)) == rt.blake3_hex(b"abc") == bytes_digest(b"abc")
    assert not file_digest(str(p)).startswith("sha256:")
    assert hashlib.sha256(b"abc").hexdigest() != file_digest(str(p))


def test_safetensors_roundtrip(rt, tmp_path):
    import safetensors.torch as st
    from comfy_gen_server_amd.runtime import checkpoint as C
    sd = {"a.weight": torch.randn(3, 4), "b": torch.arange(10, dtype=torch.int64),
          "c": torch.randn(2, 2).to(torch.bfloat16), "empty": torch.zeros(0), "h": torch.randn(5).half(),
          "f8": torch.randn(4).to(torch.float8_e4m3fn), "ué": torch.ones(2, dtype=torch.uint8)}
    meta = {"k": 'quote " and \\ backslash', "newline": "a\nb", "unicode": "é中"}
    path = str(tmp_path / "x.safetensors")
    C.save_state_dict(sd, path, meta)
    back = C.load_state_dict(path)                      # C++ reader
    ref = st.load_file(path)                            # reference reader on our file
    for k, v in sd.items():
        assert back[k].dtype == v.dtype and torch.equal(back[k].view(torch.uint8), v.view(torch.uint8)), k
        assert torch.equal(ref[k].view(torch.uint8), v.view(torch.uint8)), k
    assert C.read_metadata(path) == meta
    # a file written by the safetensors package loads through the C++ reader
    p2 = str(tmp_path / "y.safetensors")
    st.save_file({"w": torch.randn(7, 3), "i": torch.arange(4, dtype=torch.int32)}, p2, metadata={"m": "1"})
    f = rt.SafeTensorsFile(p2)
    assert sorted(f.keys()) == ["i", "w"] and f.metadata() == {"m": "1"}
    out = torch.empty(7, 3)
    f.read_into(["w"], [out.data_ptr()], 4)
    assert torch.equal(out, st.load_file(p2)["w"])


def test_safetensors_rejects_corrupt(rt, tmp_path):
    p = tmp_path / "bad.safetensors"
    hdr = b'{"t":{"dtype":"F32","shape":[4],"data_offsets":[0,64]}}'
    p.write_bytes(len(hdr).to_bytes(8, "little") + hdr + b"\0" * 16)
    with pytest.raises(Exception):
        rt.SafeTensorsFile(str(p))


def test_bpe_matches_python(rt):
    from comfy_gen_server_amd.runtime.tokenizer import CLIPTokenizer
    tok = CLIPTokenizer()
    assert tok._native is not None
    texts = ["a photo of an astronaut riding a horse on mars, highly detailed!!",
             "Ünïcödé façade — naïve café 東京 (masterpiece:1.3) [[embedding:foo]]",
             "supercalifragilisticexpialidocious antidisestablishmentarianism 1234567 x_y-z"]
    native = [tok.encode(t) for t in texts]
    tok._native = None
    python = [tok.encode(t) for t in texts]
    assert native == python
    assert native[0][:3] == [320, 1125, 539]    # "a photo of"


@pytest.mark.gpu
def test_safetensors_direct_hbm_upload(cuda, tmp_path):
    """Whole-file upload into one HBM arena (pinned double-buffered H2D) == the host reader,
    including an odd-sized uint8 tensor that leaves later tensors element-misaligned."""
    from comfy_gen_server_amd.runtime import checkpoint
    g = torch.Generator().manual_seed(0)
    sd = {"a_u8": torch.randint(0, 255, (7,), dtype=torch.uint8, generator=g),
          "b_bf16": torch.randn(33, 17, generator=g).to(torch.bfloat16),
          "c_f32": torch.randn(1000, 257, generator=g),
          "d_f16": torch.randn(5, generator=g).half(),
          "e_i64": torch.arange(9, dtype=torch.int64),
          "f_empty": torch.zeros(0, 4)}
    p = str(tmp_path / "t.safetensors")
    checkpoint.save_state_dict(sd, p)
    dev = checkpoint.load_safetensors_to_device(p, cuda)
    assert dev is not None
    for k, v in sd.items():
        assert dev[k].device.type == "cuda" and dev[k].dtype == v.dtype and dev[k].shape == v.shape
        assert torch.equal(dev[k].cpu(), v), k
    conv = checkpoint.load_safetensors_to_device(p, cuda, dtype=torch.bfloat16)
    assert conv["c_f32"].dtype == torch.bfloat16 and conv["e_i64"].dtype == torch.int64
    assert torch.equal(conv["c_f32"].cpu(), sd["c_f32"].to(torch.bfloat16))
    big = {"w": torch.randn((64 << 20) // 4 + 123, generator=g)}   # > one 64 MiB staging chunk
    p2 = str(tmp_path / "big.safetensors")
    checkpoint.save_state_dict(big, p2)
    assert torch.equal(checkpoint.load_state_dict(p2, device=cuda)["w"].cpu(), big["w"])


def test_doctor_report():
    from comfy_gen_server_amd.tools import doctor
    r = doctor.report()
    assert r["kernels_lib"] and r["kernels_missing"] == [] and r["runtime_lib"]
    assert r["distributed"]["gloo"] is True
