"""uam_path_planning_amd -- MI355X-native batched candidate-path cost evaluation for the
nomaporon/uam_path_planning hot path.

Subpackages:
  path_generation  drop-in for the reference's path_generation classes (GPU-evaluated)
  map_generation   DEM / GeoTIFF-tile ingest and the cost-raster build
Modules:
  engine     libuampath device context (torch tensors as buffers)
  batch      CandidateEvaluator: pairs x displacements -> costs + argmin, raster or analytic
  scenario   canonical Nagasaki scenario and BASELINE configs
"""
__version__ = "0.1.0"
