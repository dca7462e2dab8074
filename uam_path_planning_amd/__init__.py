"""uam_path_planning_amd -- MI355X-native batched candidate-path cost evaluation for the
nomaporon/uam_path_planning hot path.

Subpackages:
  path_generation  drop-in for the reference's path_generation classes (GPU-evaluated)
  map_generation   DEM / GeoTIFF-tile ingest, the cost-raster build, land polygons
  geo              coordinate reference systems (JGD2011 <-> plane TM) and shapefile export
Modules:
  engine       libuampath device context (torch tensors as buffers): eval_generated (pairs x
               displacements -> costs + selection, raster / analytic / volume), refine, ...
  _lib         ctypes binding of the C ABI (include/uampath.h)
  arcs         unit-arc table of the candidate generator (solver.py:103-136)
  geometry     shape compiler (polygon / ball / square -> device tables)
  distributed  pair sharding and the RCCL raster broadcast (one process per GPU)
  scenario     canonical Nagasaki scenario and BASELINE configs
  synthetic    synthetic DEM / pairs / no-fly polygons with the reference data's statistics
"""
__version__ = "0.1.0"
