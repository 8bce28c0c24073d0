class Crossover:
    def __init__(self, n_parents, n_offsprings, prob=0.9):
        self.n_parents, self.n_offsprings, self.prob = n_parents, n_offsprings, prob
