"""C-ABI surface and host-side logic.  CPU only (no compute calls into the GPU)."""
import ctypes
import re

import numpy as np
import pytest


def test_library_exports_every_declared_symbol():
    from otfuse import _lib as L
    lib = L.lib()
    declared = L.declared_symbols()
    assert len(declared) >= 10
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(L._SIGS) == set(declared), "ctypes table and header differ"


def test_version_and_workspace_queries_are_host_only():
    from otfuse import _lib as L
    lib = L.lib()
    assert lib.otf_version().decode().startswith("otfuse")
    ws = lib.otf_sinkhorn_workspace_size(4096, 4096, L.OTF_F32, 100)
    # streaming buffers (~9 vectors), the persistent engines' 4-slot sum rings, the tiled
    # engine's row exchange, the sweep engine's partial slab (256 rows of N) and the mesh
    # engine's granule slots (2 parities x 256 tiles x (4 KB column + 1.25 KB row + 256 B)),
    # the sweep engine's granule flush (256 slab rows + 16 XCC partials + 32 S slots, 8 B a
    # column, + 8 KB of registration lists)
    mesh = 2 * 256 * (4096 + 1280 + 256)
    gran = (256 + 16 + 32) * 4096 * 8 + 8192
    # the shifted kernel's offsets / initial scalings (4 vectors) and the column pass's
    # (max, sum) partials of 128 row chunks
    shift = 4 * 4096 * (4 + 2 * 128)
    assert 4 * 4096 * (9 + 16 + 256) + mesh + gran + shift < ws < 4 * 4096 * (80 + 256) + mesh + gran + shift
    # only the err log grows with max_iter (the ring replaces per-iteration buffers)
    ws_long = lib.otf_sinkhorn_workspace_size(4096, 4096, L.OTF_F32, 100000)
    assert ws_long - ws <= 8 * 100000 + 512
    # a small problem (8 row blocks) keeps a single replica
    ws_small = lib.otf_sinkhorn_workspace_size(128, 4096, L.OTF_F32, 100)
    assert ws_small < ws
    assert lib.otf_sinkhorn_workspace_size(8, 512, L.OTF_F64, 2000) > 8 * 512 * 7
    assert lib.otf_feature_cost_workspace_size(8, 8, 512, 512) >= 8 * (8 * 512)


def test_abi_structs_and_enums_match_header():
    from otfuse import _lib as L
    src = open(L.HEADER_PATH).read()
    assert ctypes.sizeof(L.SinkhornOpts) == 56   # 2 doubles + 9 int32, 8-aligned
    # otf_sinkhorn_info: the int32 fields of the header, in order, are INFO_FIELDS
    import re
    hdr = open(L.HEADER_PATH).read()
    body = hdr[:hdr.index("} otf_sinkhorn_info;")]
    body = body[body.rindex("typedef struct"):]
    fields = re.findall(r"int32_t\s+(\w+);", body)
    assert tuple(fields) == L.INFO_FIELDS and L.INFO_INT32S == len(fields)
    for name, val in [("OTF_F32", 0), ("OTF_F64", 1), ("OTF_F16", 2), ("OTF_BF16", 3),
                      ("OTF_ENGINE_SWEEP", 4), ("OTF_RED_SUM", 0), ("OTF_RED_MAX", 1),
                      ("OTF_FLAVOR_POT", 0),
                      ("OTF_FLAVOR_OTT", 1),
                      ("OTF_SK_CONVERGED", 1), ("OTF_SK_MAX_ITER", 2),
                      ("OTF_SK_NUMERICAL_BREAK", 3)]:
        m = re.search(rf"\b{name}\s*=\s*(-?\d+)", src)
        assert m and int(m.group(1)) == val, name


def test_invalid_arguments_are_rejected_without_a_gpu():
    """Argument validation runs before any HIP call."""
    from otfuse import _lib as L
    lib = L.lib()
    opts = L.SinkhornOpts(reg=0.1, stop_thr=0.0, max_iter=10, check_every=10, flavor=0,
                          err_squared=0, sync_every=0, engine=0)
    rc = lib.otf_sinkhorn(None, None, None, 0, 0, 0, L.OTF_F32, None, ctypes.byref(opts), None,
                          None, None, 0, 0, None, None, None, 0, None)
    assert rc == L.OTF_EINVAL
    assert lib.otf_cost_pairwise(None, 0, None, 0, 4, 4, 4, 0, 0, None, 4, None, None) == L.OTF_EINVAL
    assert lib.otf_gemm_f32(None, 1, 1, None, 1, 1, None, 1, 1, 1, 1, 1.0, 0.0, None) == L.OTF_EINVAL
    # fp16 cost entry point: bad dtypes and an undersized workspace are argument errors
    ws = lib.otf_cost_ex_workspace_size(64, 64, 32, L.OTF_F16)
    assert ws < lib.otf_cost_ex_workspace_size(64, 64, 32, L.OTF_F32)  # no lo images
    buf = ctypes.create_string_buffer(16)
    p = ctypes.cast(buf, ctypes.c_void_p)
    assert lib.otf_cost_pairwise_ex(p, 32, p, 32, L.OTF_F64, 64, 64, 32, 0, 0, p, 64, L.OTF_F16,
                                    None, None, p, ws, None) == L.OTF_EINVAL
    assert lib.otf_cost_pairwise_ex(p, 32, p, 32, L.OTF_F16, 64, 64, 32, 0, 0, p, 64, L.OTF_F16,
                                    None, None, p, ws - 1, None) == L.OTF_EINVAL


def test_group_features_by_label_mirrors_reference():
    from otfuse.fusion import group_features_by_label
    y = np.array([1, 0, 1, 1, 0, 2])
    p = np.arange(12, dtype=np.float32).reshape(6, 2)
    g = group_features_by_label(y, p, max_samples_per_label=2)
    assert list(g.keys()) == [0, 1, 2]
    np.testing.assert_array_equal(g[1], p[[0, 2]])
    np.testing.assert_array_equal(g[0], p[[1, 4]])
    np.testing.assert_array_equal(g[2], p[[5]])
    g2 = group_features_by_label(y, p)
    assert g2[1].shape == (3, 2)


def test_mdict_to_matrix_and_block_diag(orc):
    from otfuse.perturbot import mdict_to_matrix
    from otfuse.pot import block_diag_ts
    rng = np.random.default_rng(0)
    xd = {1: rng.random((3, 2)), 0: rng.random((2, 2))}
    yd = {1: rng.random((4, 2)), 0: rng.random((2, 2))}
    ts = {0: rng.random((2, 2)), 1: rng.random((3, 4))}
    # nojax: sorted label order
    np.testing.assert_array_equal(block_diag_ts(ts, xd, yd), orc.block_diag_ts(ts, xd, yd))
    B = block_diag_ts(ts, xd, yd)
    np.testing.assert_array_equal(B[:2, :2], ts[0])
    np.testing.assert_array_equal(B[2:, 2:], ts[1])
    # perturbot: insertion order of data[0] through label masks
    src = np.concatenate([np.ones(xd[k].shape[0]) * k for k in xd])
    tgt = np.concatenate([np.ones(yd[k].shape[0]) * k for k in xd])
    Mt = mdict_to_matrix(ts, src, tgt)
    np.testing.assert_array_equal(Mt[:3, :4], ts[1])
    np.testing.assert_array_equal(Mt[3:, 4:], ts[0])
    assert Mt[:3, 4:].sum() == 0


def test_synthetic_inputs_are_seeded_and_structured():
    from otfuse.synthetic import paired_embeddings
    X1, Y1, l1 = paired_embeddings(64, 32, seed=9)
    X2, Y2, l2 = paired_embeddings(64, 32, seed=9)
    np.testing.assert_array_equal(X1, X2)
    np.testing.assert_array_equal(l1, l2)
    assert X1.dtype == np.float32 and (X1 >= 0).all()
    # paired: a subject's MRI embedding is closer to its own PET embedding's latent
    # neighbourhood than to a random subject's (structure, not iid noise)
    c = np.corrcoef(X1.reshape(-1), Y1.reshape(-1))[0, 1]
    assert np.isfinite(c)


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from otfuse import _lib as L
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.OtfError):
        L.lib()


def test_engine_enum_matches_header():
    """The Python engine table (otfuse._lib.ENGINES) and the header's otf_engine enum agree,
    including the gather and mesh engines (host-only: parses include/otfuse.h)."""
    import os
    import re
    from otfuse import _lib as L
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "otfuse.h")).read()
    body = hdr[hdr.index("typedef enum {\n    OTF_ENGINE_AUTO"):]
    body = body[:body.index("} otf_engine;")]
    enum = {m.group(1).lower(): int(m.group(2))
            for m in re.finditer(r"OTF_ENGINE_([A-Z]+)\s*=\s*(\d+)", body)}
    assert enum == L.ENGINES
    assert {"gather", "mesh"} <= set(enum)
