"""CPU oracle for the BlueSky CD / MVP / kinematics hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``bluesky_amd/`` imports this
package: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker
(or the timed CPU baseline), never as the product path.

The modules restate the reference algorithms in numpy, operation for
operation and in the reference's evaluation order, so that on the same
numpy build they are bit-for-bit equal to the reference (pinned by the
golden fixtures in ``tests/golden/``, which were captured by importing the
reference itself in the build container, see ``tools/make_golden.py``).

* ``statebased`` -- ``StateBasedCD.detect`` + ``geo.qdrdist_matrix``
  (reference ``bluesky/traffic/asas/StateBasedCD.py:7-103``,
  ``bluesky/tools/geo.py:32-54,110-162``), row-chunked so that it runs at
  N where the reference's N x N temporaries do not fit.
* ``mvp`` -- ``MVP.resolve`` / ``MVP.MVP`` / ``MVP.prioRules``
  (``bluesky/traffic/asas/MVP.py:14-300``) with a dict index instead of
  ``list.index``.
* ``kinematics`` -- ``Traffic.UpdateAirSpeed/UpdateGroundSpeed/
  UpdatePosition`` (``bluesky/traffic/traffic.py:425-483``) and the ISA
  helpers they call (``bluesky/tools/aero.py:62-147``).
* ``step`` -- the build-defined synthetic sim step
  composed from the three above.
"""
