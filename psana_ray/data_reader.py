from psana_ray_amd.data_reader import DataReader, DataReaderError, EndOfStream  # noqa: F401
