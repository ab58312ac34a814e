"""Host logic of the `methods` driver (no GPU): the method file, pair input
columns, GenomePairList grouping, previous-results validation and the
correlation statistics (MethodTableProcessor.java:149-221,339-378)."""
import io

import numpy as np
import pytest
import scipy.stats


class _NoCtx:
    """Stands in for a device context: nothing here touches the device."""


def _methods(spec):
    from gdist import methods as M
    return M.read_method_file(io.StringIO("type\tparms\n" + spec), _NoCtx())


def test_method_file_and_headers():
    from gdist.processors import ParseFailureException
    ms = _methods("prot\tK=8\nkmer\tK=21\nPROT\t\n")
    assert [str(m) for m in ms] == ["PROT_K8", "KMER_K21", "PROT_K8"]
    with pytest.raises(ParseFailureException):
        _methods("blast\t\n")
    with pytest.raises(ParseFailureException):
        _methods("prot\tW=3\n")
    with pytest.raises(ParseFailureException):
        _methods("kmer\tK=1\n")


def test_pairs_columns_and_grouping():
    from gdist import methods as M
    tsv = "a\tgenome_id\tother\n1\tg1\tg2\n2\tg3\tg1\n3\tg1\tg4\n4\tg3\tg2\n"
    assert M.read_pairs(io.StringIO(tsv), "genome_id", "3") == [("g1", "g2"), ("g3", "g1"), ("g1", "g4"),
                                                                ("g3", "g2")]
    with pytest.raises(IOError):
        M.read_pairs(io.StringIO(tsv), "nosuch", "2")
    assert M.group_pairs([("g1", "g2"), ("g3", "g1"), ("g1", "g4")]) == [("g1", ["g2", "g4"]), ("g3", ["g1"])]


def test_previous_results_validation():
    from gdist import methods as M
    ms = _methods("prot\tK=8\nkmer\tK=21\n")
    head = "id1\tname1\tid2\tname2\ttax_group\tPROT_K8\tKMER_K21\n"
    old = M.load_previous(io.StringIO(head + "a\tA\tb\tB\tgenus\t0.5\t9.5E-4\nb\tB\tc\tC\tnone\t1.0\tNaN\n"), ms)
    assert old[("a", "b")] == [0.5, 9.5e-4]
    assert old[("b", "c")][0] == 1.0 and np.isnan(old[("b", "c")][1])
    with pytest.raises(IOError, match="Method 1 does not match"):
        M.load_previous(io.StringIO(head), _methods("prot\tK=8\nkmer\tK=13\n"))
    with pytest.raises(IOError, match="wrong number of columns"):
        M.load_previous(io.StringIO(head), _methods("prot\tK=8\n"))


def test_statistics_against_scipy():
    from gdist import methods as M
    from gdist.javafmt import java_format_f
    rng = np.random.default_rng(1)
    a = rng.random(40)
    b = np.round(a * 0.7 + rng.random(40) * 0.3, 2)               # ties in b
    ms = _methods("prot\tK=8\nkmer\tK=21\n")
    out = io.StringIO()
    M.write_statistics(out, ms, np.stack([a, b], 1).tolist())
    lines = out.getvalue().splitlines()
    assert lines[0] == "method1\tmethod2\tPearson\tKendall\tSpearman\tvariation\tIQR"
    assert [l.split("\t")[:2] for l in lines[1:]] == [["KMER_K21", "PROT_K8"], ["PROT_K8", "KMER_K21"]]
    vals = lines[1].split("\t")[2:]
    exp = [scipy.stats.pearsonr(a, b)[0], scipy.stats.kendalltau(a, b)[0], scipy.stats.spearmanr(a, b)[0]]
    assert vals[:3] == [java_format_f(x, 8, 4) for x in exp]
