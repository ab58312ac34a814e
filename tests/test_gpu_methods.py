"""BASELINE config C1 through the Measurer plugin path:
10 synthetic genomes of 100 kbp, each with its proteome as one 33,333-aa
protein, protein k=8 (and contig DNA k=21 as a second method), driven as
MethodTableProcessor.runPipeline does (MethodTableProcessor.java:234-308):
DistanceMethod.create / parseParmString / toString headers / getMeasurer /
concurrent getDistance from 8 threads / Double.toString rows / --previous
reuse with header validation. Expectations come from the pure-Python string
restatement (oracle/pyref.py) and Java Double.toString (pyref.java_double_str)."""
import concurrent.futures as cf
import io
import itertools

import numpy as np
import pytest

import pyref

pytestmark = pytest.mark.gpu

N = 10


def _genomes():
    from gdist import synth
    from gdist.processors import Genome
    dna = synth.genomes(N, 100_000, 0.05, 1)
    prot = synth.genomes(N, 33_333, 0.10, 1, protein=True)
    ranks = ("superkingdom", "phylum", "class", "order", "family", "genus", "species")
    out = {}
    for i in range(N):
        # lineages diverge at different depths (genome i's taxon at rank d is
        # i >> (6 - d)); the last genome has no lineage ("none")
        lin = {r: f"{r}-{i >> (6 - d)}" for d, r in enumerate(ranks)} if i < N - 1 else {}
        gid = f"{83333 + i}.{i + 1}"
        out[gid] = Genome(gid, f"Synthetic genome {i}", [bytes(dna[i]).decode()], [bytes(prot[i]).decode()], lin)
    return out


def _expected_lines(genomes, pairs, ks=(("prot", 8), ("kmer", 21))):
    from gdist.methods import TaxonDistanceMethod
    tax = TaxonDistanceMethod()
    sets = {}
    for gid, g in genomes.items():
        sets[("prot", gid)] = pyref.kmer_set("\0".join(g.proteins), 8, pyref.PROT)
        sets[("kmer", gid)] = pyref.kmer_set("\0".join(g.contigs), 21, pyref.DNA)
    lines = []
    for a, b in pairs:
        ds = [pyref.java_double_str(pyref.set_distance(sets[(t, a)], sets[(t, b)])) for t, _ in ks]
        grp = tax.getGroupingLevel(TaxonDistanceMethod.Analysis(genomes[a]), TaxonDistanceMethod.Analysis(genomes[b]))
        lines.append("\t".join([a, genomes[a].name, b, genomes[b].name, grp] + ds))
    return lines


def _methods(ctx, spec="prot\tK=8\nkmer\tK=21\n"):
    from gdist import methods as M
    return M.read_method_file(io.StringIO("type\tparms\n" + spec), ctx)


def test_c1_method_table_bit_exact(ctx, tmp_path):
    from gdist import methods as M
    genomes = _genomes()
    ids = list(genomes)
    pairs = list(itertools.combinations(ids, 2))
    rng = np.random.default_rng(3)
    pairs = [pairs[i] for i in rng.permutation(len(pairs))]          # input order: groups interleaved
    tsv = "genome1\tgenome2\n" + "".join(f"{a}\t{b}\n" for a, b in pairs)
    read = M.read_pairs(io.StringIO(tsv), "1", "2")
    assert read == pairs
    methods = _methods(ctx)
    assert [str(m) for m in methods] == ["PROT_K8", "KMER_K21"]
    out, stats = io.StringIO(), io.StringIO()
    counts = M.method_table(read, methods, genomes, out, stats=stats, threads=8)
    assert counts == {"pairs": 45, "computed": 45, "reused": 0}
    lines = out.getvalue().splitlines()
    assert lines[0] == "id1\tname1\tid2\tname2\ttax_group\tPROT_K8\tKMER_K21"
    grouped = [(a, b) for a, bs in M.group_pairs(pairs) for b in bs]   # GenomePairList.prepare order
    assert lines[1:] == _expected_lines(genomes, grouped)
    assert {l.split("\t")[4] for l in lines[1:]} >= {"none", "genus", "family", "order", "class"}
    st = stats.getvalue().splitlines()
    assert st[0] == "method1\tmethod2\tPearson\tKendall\tSpearman\tvariation\tIQR"
    assert [l.split("\t")[:2] for l in st[1:]] == [["KMER_K21", "PROT_K8"], ["PROT_K8", "KMER_K21"]]
    # the statistics' values against scipy's (commons-math Pearson, Kendall
    # tau-b, Spearman on average ranks; MethodTableProcessor.java:364-366),
    # over the table's distance columns in pair order; %8.4f fields
    from scipy import stats as sst
    d1 = np.array([float(l.split("\t")[5]) for l in lines[1:]])
    d2 = np.array([float(l.split("\t")[6]) for l in lines[1:]])
    exp = (sst.pearsonr(d1, d2)[0], sst.kendalltau(d1, d2, variant="b")[0], sst.spearmanr(d1, d2)[0])
    for row in st[1:]:
        got = [float(x) for x in row.split("\t")[2:5]]
        assert np.allclose(got, exp, atol=5.1e-5, rtol=0), (row, exp)

    # --previous: every pair reused (getDistance must not run), same rows
    prev = tmp_path / "prev.tbl"
    prev.write_text(out.getvalue())
    methods2 = _methods(ctx)
    old = M.load_previous(prev.read_text().splitlines(True), methods2)
    assert len(old) == 45
    for m in methods2:
        m.getDistance = None                                        # would raise if called
        m.prefetch = None
    out2 = io.StringIO()
    counts2 = M.method_table(read, methods2, genomes, out2, previous=old, threads=8)
    assert counts2 == {"pairs": 45, "computed": 0, "reused": 45}
    assert out2.getvalue() == out.getvalue()
    # a mismatched method configuration is rejected (MethodTableProcessor.java:198-203)
    with pytest.raises(IOError, match="Method 0 does not match"):
        M.load_previous(prev.read_text().splitlines(True), _methods(ctx, "prot\tK=9\nkmer\tK=21\n"))
    with pytest.raises(IOError, match="wrong number of columns"):
        M.load_previous(prev.read_text().splitlines(True), _methods(ctx, "prot\tK=8\n"))
    # a partial previous file: only the missing pairs are computed
    keep = dict(list(old.items())[:20])
    out3 = io.StringIO()
    counts3 = M.method_table(read, _methods(ctx), genomes, out3, previous=keep, threads=8)
    assert counts3 == {"pairs": 45, "computed": 25, "reused": 20}
    assert out3.getvalue() == out.getvalue()


def test_measurer_concurrent_get_distance(ctx):
    """getDistance from 8 threads at once (the ForkJoin calls of :275), no
    prefetch: every value bit-exact against the string restatement."""
    from gdist.methods import DistanceMethod
    genomes = _genomes()
    ids = list(genomes)
    m = DistanceMethod.create("prot", ctx)
    m.parseParmString("K=8")
    meas = {a: m.getMeasurer(genomes[a]) for a in ids[:3]}
    jobs = [(a, b) for a in ids[:3] for b in ids]
    with cf.ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda p: m.getDistance(meas[p[0]], genomes[p[1]]), jobs))
    ks = {g: pyref.kmer_set(genomes[g].proteins[0], 8, pyref.PROT) for g in ids}
    for (a, b), d in zip(jobs, got):
        assert pyref.java_double_str(d) == pyref.java_double_str(pyref.set_distance(ks[a], ks[b])), (a, b)
    with pytest.raises(ValueError):
        DistanceMethod.create("nosuch", ctx)
    with pytest.raises(ValueError):
        m.parseParmString("K=1")
