from psana_ray_amd.producer import (initialize_queue, initialize_ray, main, parse_arguments,  # noqa: F401
                                    produce_data)

if __name__ == "__main__":
    import sys

    sys.exit(main())
