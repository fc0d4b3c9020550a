from psana_ray_amd.shared_queue import Queue, create_queue  # noqa: F401
