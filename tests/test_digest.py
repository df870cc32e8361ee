"""CPU: the product's host-side digest fold equals the oracle's definition."""
import numpy as np

from lifeapi_amd.digest import batch_digest, combine


def test_batch_digest_matches_oracle(port):
    x = port.fill(3000, seed=21, first_universe=777)
    h = port.hashes(x)
    assert batch_digest(h, 777) == port.digest(h, 777)
    assert combine([batch_digest(h[:1234], 777), batch_digest(h[1234:], 777 + 1234)]) == \
        batch_digest(h, 777)
    assert batch_digest(h.view(np.int64), 777) == port.digest(h, 777)
