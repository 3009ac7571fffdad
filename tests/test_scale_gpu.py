"""Parity at BASELINE scale through digests (tests/golden/make_digests.py):
C4 (20k nodes x 500k tasks, BASELINE configs[3]) and a saturated C3-size
session whose per-task requests fill the cluster mid-cycle, so the default
K = 8192 batches are cut by unpredicted failures and the ordering engine is
rolled back and replayed (allocate.go:105-171: a task that fits nowhere
leaves its job unpushed). Bit-exact decision log, binds, node and job states;
shares within 1e-12 relative."""
import pytest

from helpers import compare_digests, digest_outputs, load_golden

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import synth  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402

GEN = {"c4": lambda: synth.config_fixture(4), "saturated": lambda: synth.saturated_config()}


@pytest.fixture(scope="module")
def saturated():
    return GEN["saturated"]()


@pytest.mark.parametrize("opts", [{}, {"full_scan": 1}, {"batch_tasks": 2048, "candidates": 8},
                                  {"shards": 4}])
def test_saturated_parity(saturated, opts):
    ref = load_golden("digest_saturated.json")
    got, ssn = run_fixture(saturated, opts)
    st = ssn.stats()
    ssn.close()
    compare_digests(ref, digest_outputs(got))
    assert st.task_evaluations == ref["evaluated"]
    if not opts:
        # the speculation machinery really ran: unpredicted failures cut
        # batches and the predictor restarted from the truth engine at the cut
        assert st.mispredictions > 0, st.mispredictions


@pytest.mark.parametrize("env", ["KBG_NO_CUT_REUSE", "KBG_HOST_FITDELTA"])
def test_saturated_ab_paths(saturated, env, monkeypatch):
    """The saturated session with the cut-time list reuse turned off (every
    cut rescans) and with FitError counted on the host instead of by
    kbg_fitdelta_kernel: the same digest as the default paths, so parity does
    not hinge on either."""
    ref = load_golden("digest_saturated.json")
    monkeypatch.setenv(env, "1")
    got, ssn = run_fixture(saturated)
    st = ssn.stats()
    ssn.close()
    compare_digests(ref, digest_outputs(got))
    if env == "KBG_NO_CUT_REUSE":
        assert st.reused_batches == 0, st.reused_batches


@pytest.mark.slow
def test_config4_parity():
    ref = load_golden("digest_c4.json")
    got, ssn = run_fixture(GEN["c4"]())
    st = ssn.stats()
    ssn.close()
    compare_digests(ref, digest_outputs(got))
    assert st.task_evaluations == ref["evaluated"]
