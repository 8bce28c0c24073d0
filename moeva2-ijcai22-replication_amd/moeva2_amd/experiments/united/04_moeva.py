"""``python -m moeva2_amd.experiments.united.04_moeva -c config/moeva.yaml -c <project>.yaml
-p seed=42 -p budget=100 -j '{"eps_list":[0.2]}'`` -- same command line as
src/experiments/united/04_moeva.py (see moeva_run.py)."""
from moeva2_amd.experiments.united.moeva_run import main

if __name__ == "__main__":
    main()
