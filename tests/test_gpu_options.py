"""Tuning options live in the context (gdist_ctx_set_option), never in the
environment: a JNI host with a different environment runs the same kernels
(callers sharing one context, MethodTableProcessor.java:275)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_gpu_box_library_matches_tree():
    """On the GPU box: the library these tests load was built from the
    sources of the snapshot they run from."""
    from gdist import _lib
    _lib.check_build()


def test_option_roundtrip_and_errors(ctx):
    import gdist
    names = gdist.option_names()
    for n in ("rare_t", "rare_kernel", "bitset_diag", "sparse", "sparse_zmax", "sketch_k", "reps_block",
              "locus_order", "guides", "sparse_part_budget", "sparse_groups", "sketch_v2", "sketch_phase",
              "sketch_cap", "sketch_ring", "sketch_wait", "sparse_xcd", "time_kernels",
              "rare_u16", "rare_rows_threads", "rare_direct", "split_build", "variant_c16", "variant_split", "rare_group", "variant_short", "variant_bits", "bitset_mfma_store", "variant_pack_keyless", "epilogue_rows", "bitset_mfma_raw", "serial_step", "dense_first", "reps_split", "rare_c16", "sort_radix", "bitset_mfma", "bitset_mfma_km", "bitset_mfma_group", "bitset_mfma_ns", "bitset_mfma_splits", "sparse_mt", "sparse_sun", "sparse_dyn", "sparse_diag22", "sparse_rpart22", "pack_code_sort", "variant", "variant_dmin", "range_summary"):
        assert n in names
    # round 3: superseded kernel variants and the result-changing ablation
    # switch are gone; every remaining option preserves results
    for n in ("sparse_abl", "sparse_kernel", "bitset_kernel", "sparse_shape", "sparse_occ", "fold_dense_words",
              "sketch_sw", "sketch_map", "sketch_split"):
        assert n not in names
    c = gdist.Context(0)
    try:
        assert c.option("sparse") is None
        c.set_option("sparse", 0)
        assert c.option("sparse") == 0
        with c.options(sparse=1, rare_t=7):
            assert c.option("sparse") == 1 and c.option("rare_t") == 7
        assert c.option("sparse") == 0 and c.option("rare_t") is None
        c.set_option("sparse", None)
        assert c.option("sparse") is None
        with pytest.raises(ValueError):
            c.set_option("no_such_option", 1)
    finally:
        c.close()


def test_environment_does_not_change_kernels(monkeypatch):
    """GDIST_* variables in the process environment are ignored by the
    library: the sparse split and the rare threshold follow the context."""
    import gdist
    from gdist import synth
    seqs = [bytes(r) for r in synth.genomes(160, 20000, 0.003, 7)]
    monkeypatch.setenv("GDIST_SPARSE", "0")
    monkeypatch.setenv("GDIST_RARE_T", "3")
    c = gdist.Context(0)
    try:
        a = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, c)
        a.build_bitsets()
        t_env = a.rare_info()[0]
        monkeypatch.delenv("GDIST_RARE_T")
        a.build_bitsets()
        assert a.rare_info()[0] == t_env, "GDIST_RARE_T in the environment must not change T"
        monkeypatch.setenv("GDIST_RARE_T", "3")
        c.set_option("sparse_zmax", 100000)           # force the split through the context
        b = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, c)
        b.build_bitsets()
        assert b.sparse_info()[0] > 0, "GDIST_SPARSE=0 in the environment must not switch the split off"
        c.set_option("sparse", 0)
        d = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, c)
        d.build_bitsets()
        assert d.sparse_info()[0] == 0
        c.set_option("rare_t", 5)
        d.build_bitsets()
        assert d.rare_info()[0] == 5
        I1, _ = b.matrix(upper=True, method=gdist.METHOD_BITSET)
        I2, _ = d.matrix(upper=True, method=gdist.METHOD_BITSET)
        iu = np.triu_indices(len(seqs), 1)
        assert np.array_equal(I1[iu], I2[iu])
    finally:
        c.close()            # frees a, b, d first (a collection must not outlive its context)


def test_plan_follows_options(ctx, opts):
    """A region's cached launch plan is keyed by the options it reads: turning
    option sparse_rare off on the same collection and region rebuilds the plan
    (the rare tier then runs as its own kernel: 2 launches instead of the fused
    step's 1), and every call stays oracle-exact."""
    import gdist
    import oracle
    from gdist import synth
    seqs = [bytes(r) for r in synth.genomes(300, 20000, 0.003, 11)]
    sets = gdist.KmerSets.from_sequences(seqs, 21, gdist.KmerType.DNA, 0, ctx)
    sets.build_bitsets()
    assert sets.sparse_info()[0] > 0 and sets.rare_info()[1] > 0
    off, codes = oracle.pack(seqs, 21, 0, 0)
    eI, eD = oracle.matrix(off, codes, 0, 300, 0, 300, flags=0x100)
    iu = np.triu_indices(300, 1)
    launches = []
    for rare in (None, 0, None):
        opts(sparse_rare=rare)
        I, D = sets.matrix(upper=True, method=gdist.METHOD_BITSET)
        assert np.array_equal(I[iu], eI[iu]) and np.array_equal(D[iu].view(np.uint64), eD[iu].view(np.uint64))
        launches.append(ctx.last_timing()[2])
    assert launches == [1, 2, 1], launches
