"""Import-path compatibility for users of carbonscott/psana-ray: ``from psana_ray.data_reader
import DataReader`` keeps working; everything is implemented in :mod:`psana_ray_amd`."""
