"""GPU, BASELINE configs[2] (C3) at its stated shape: 1M nodes x 10M pods
sharded over 8 engine ranks on one MI355X (~125k nodes, ~1.25M pods each),
initial tick + a 1M-delete / 1M-create churn tick + a steady tick, against
the single-rank oracle of the whole fleet (tests/c3_common.py)."""
import pytest

from c3_common import run_c3

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(1100)
def test_eight_rank_c3_initial_and_churn_ticks():
    run_c3(8, 1_000_000, 1_000_000, "engine")
