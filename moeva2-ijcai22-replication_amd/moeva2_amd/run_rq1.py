"""src/run_rq1.py (MoEvA part): see run_rq.py."""
from moeva2_amd.run_rq import main

if __name__ == "__main__":
    main("rq1")
