"""src/run_rq2.py (MoEvA part): see run_rq.py."""
from moeva2_amd.run_rq import main

if __name__ == "__main__":
    main("rq2")
