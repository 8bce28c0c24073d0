class NonDominatedSorting:
    def __init__(self, *a, **k):
        pass
