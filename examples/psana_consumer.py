"""Reference-style consumer (examples/psana_consumer.py of carbonscott/psana-ray), fixed:

Launch a producer (it hosts the rendezvous store unless `psana-ray-server` runs):
    mpirun -n 4 psana-ray-producer --exp mfxl1038923 --run 58 --detector_name epix10k2M --queue_size 400

Launch consumers (same defaults as the producer, so no flags are needed):
    python psana_consumer.py 0

Items carry 4 fields [rank, idx, data, photon_energy]; the stream ends with EndOfStream (a
DataReaderError), so this loop terminates instead of polling forever.
"""
import signal
import sys
import time

from psana_ray.data_reader import DataReader, DataReaderError, EndOfStream


def signal_handler(sig, frame):
    print("Ctrl+C pressed. Shutting down...")
    sys.exit(0)


def consume_data(consumer_id):
    with DataReader(consumer_id=consumer_id) as reader:
        while True:
            try:
                result = reader.read(timeout=1.0)
                if result is not None:
                    rank, idx, data, photon_energy = result
                    print(f"Consumer {consumer_id} processed: rank={rank} | idx={idx} | shape={tuple(data.shape)}")
                else:
                    print(f"Consumer {consumer_id} waiting for data...")
            except EndOfStream:
                print(f"Consumer {consumer_id}: end of stream")
                break
            except DataReaderError as e:
                print(f"DataReader error: {e}")
                print("Queue actor is dead. Exiting...")
                break
            except Exception as e:
                print(f"Error in consume_data: {e}")
                time.sleep(1)


if __name__ == "__main__":
    signal.signal(signal.SIGINT, signal_handler)
    consumer_id = int(sys.argv[1]) if len(sys.argv) > 1 else None
    consume_data(consumer_id)
