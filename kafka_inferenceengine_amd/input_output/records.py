"""Per-band observation records (plug-in point L1), defined once.

Field orders follow the reference: ``MOD09_data`` / ``BHR_data``
(``observations.py:69-72``), ``S2MSIdata`` (``Sentinel2_Observations.py:82-83``),
``SARdata`` (``Sentinel1_Observations.py:26-27``).  Every reader imports them
from here, so ``isinstance`` checks and pickles agree across modules.
"""
from __future__ import annotations

from collections import namedtuple

MOD09_data = namedtuple("MOD09_data", "reflectance mask uncertainty obs_op sza vza raa")
BHR_data = namedtuple("BHR_data", "observations mask uncertainty metadata emulator")
S2MSIdata = namedtuple("S2MSIdata", "observations uncertainty mask metadata emulator")
SARdata = namedtuple("SARdata", "observations uncertainty mask metadata emulator")
ObsData = namedtuple("ObsData", "observations uncertainty mask metadata emulator")
