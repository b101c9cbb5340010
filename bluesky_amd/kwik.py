"""Opt-in flat-earth ("KWIK") conflict detection on MI355X.

``detect(ownship, intruder, RPZ, HPZ, tlookahead)`` with the StateBased
contract (``StateBasedCD.py:7-103``), where ``geo.kwikqdrdist_matrix``
(``geo.py:347-363``: equirectangular distance with the mean-latitude cosine,
radius 6 371 000 m, bearing in [0, 360)) replaces ``geo.qdrdist_matrix``.
Its distance is in metres although the docstring says nm, so it is handed to
the detector divided by ``nm`` (StateBasedCD multiplies by ``nm``,
``StateBasedCD.py:22``): this is the reference's own detect with the geo
function swapped, which is how ``tools/make_golden.py`` captures the KWIK
golden vectors.

Register with ``ASAS.addCDMethod('GPUKWIK', bluesky_amd.kwik)`` (``asas.py:49-51``).
"""
from . import statebased


def detect(ownship, intruder, RPZ, HPZ, tlookahead, with_dcpa=False):
    """Flat-earth StateBased detect (8-tuple; 9-tuple with ``with_dcpa=True``)."""
    return statebased.detect(ownship, intruder, RPZ, HPZ, tlookahead, with_dcpa=with_dcpa, kwik=True)
