"""Input/output: synthetic sensors, streaming ingest, writers, checkpoints, TIFF."""
from .checkpoint import CheckpointManager  # noqa: F401
from .geo import (Polygon, find_overlap_raster_feature, parse_crs, rasterize_polygons,  # noqa: F401
                  raster_extent_feature, read_geojson_polygons)
from .modis import Kernels, MOD09_ObservationsKernels, SynergyKernels  # noqa: F401
from .observations import ArrayObservations, BHRObservationsTest, bhr_uncertainty, get_modis_dates  # noqa: F401
from .output import DeviceOutput, KafkaOutput, KafkaOutputMemory  # noqa: F401
from .synthetic import (MultiSensorObservations, SyntheticBHRObservations, SyntheticObservations,  # noqa: F401
                        SyntheticIdentityObservations, SyntheticOLCIObservations, SyntheticS1Observations,
                        SyntheticS2Observations)
from .tiff import read_tiff, read_tiff_window, tiff_info, write_tiff  # noqa: F401
from .utils import find_overlap, get_chunks, raster_extent, reproject_image  # noqa: F401
