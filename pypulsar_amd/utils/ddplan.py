"""Dedispersion planner: the DM-trial grid the batched sweep executes.

Restates the planning algorithm of ``utils/DDplan2b.py`` (Observation 50-99,
DDstep 102-199, DDplan 202-290, calc_min_smearing 292-333, guess_DMstep
438-447) with the same arithmetic, so the generated grids (loDM, dDM,
numDMs, downsamp, dsubDM, DMs_per_prepsub, numprepsub, work fractions) are
identical to the reference's (pinned by tests/golden).  Printing follows
``DDplan.__str__`` (DDplan2b.py:424-435); plotting is out of scope.

The reference has no executor for a plan; ``pypulsar_amd.sweep.execute_plan``
is the new one (per step: downsample, optional subband pass per call at
``loDM + (k + 0.5) * dsubDM`` -- PRESTO's convention -- then the DM sweep).
"""
import numpy as np

from ..delays import dm_smear, guess_DMstep

ALLOW_DMSTEPS = (0.01, 0.02, 0.03, 0.05, 0.1, 0.2, 0.3, 0.5, 1.0,
                 2.0, 3.0, 5.0, 10.0, 20.0, 30.0, 50.0, 100.0, 200.0, 300.0)
MAX_DOWNFACTOR = 64
FF = 1.2          # softening of "equal time scales"
SMEARFACT = 2.0   # allowed single-channel smearing relative to the rest


class Observation(object):
    """Observation parameters (DDplan2b.py:50-99). dt in s, fctr/BW in MHz."""

    def __init__(self, dt, fctr, BW, numchan, numsamp=0):
        self.dt = dt
        self.fctr = fctr
        self.BW = BW
        self.numchan = numchan
        self.chanwidth = BW / numchan
        self.numsamp = numsamp
        self.allow_factors = self._downfactors()

    def _downfactors(self):
        if self.numsamp:
            return [int(f) for f in range(1, MAX_DOWNFACTOR + 1) if self.numsamp % f == 0]
        return [2 ** i for i in range(int(np.log2(MAX_DOWNFACTOR)) + 1)]

    # name kept from the reference API
    get_allow_downfactors = _downfactors

    def gen_ddplan(self, loDM, hiDM, numsub=0, resolution=0.0, verbose=False):
        return DDplan(loDM, hiDM, self, numsub, resolution, verbose)


class DDstep(object):
    """One block of constant downsampling and DM step (DDplan2b.py:102-199)."""

    def __init__(self, ddplan, downsamp, loDM, dDM, numDMs=0, numsub=0, smearfact=2.0):
        obs = ddplan.obs
        self.ddplan = ddplan
        self.downsamp = downsamp
        self.loDM = loDM
        self.dDM = dDM
        self.numsub = numsub
        self.BW_smearing = dm_smear(dDM * 0.5, obs.BW, obs.fctr)
        self.numprepsub = 0
        if numsub:
            # largest even number of DMs per subband pass whose subband
            # smearing stays below 0.8 x the other contributions
            per = 2
            limit = 0.8 * min(self.BW_smearing, obs.dt * self.downsamp)
            while dm_smear((per + 2) * dDM * 0.5, obs.BW / numsub, obs.fctr) <= limit:
                per += 2
            self.dsubDM = per * dDM
            self.DMs_per_prepsub = per
            self.sub_smearing = dm_smear(self.dsubDM * 0.5, obs.BW / self.numsub, obs.fctr)
        else:
            self.dsubDM = dDM
            self.sub_smearing = 0.0
        cross_DM = min(self.DM_for_smearfact(smearfact), ddplan.hiDM)
        if numDMs == 0:
            self.numDMs = int(np.ceil((cross_DM - self.loDM) / self.dDM))
            if numsub:
                self.numprepsub = int(np.ceil(self.numDMs * self.dDM / self.dsubDM))
                self.numDMs = self.numprepsub * self.DMs_per_prepsub
        else:
            self.numDMs = numDMs
        self.hiDM = loDM + self.numDMs * dDM
        self.DMs = np.arange(self.numDMs, dtype='d') * self.dDM + self.loDM
        self.chan_smear = dm_smear(self.DMs, obs.chanwidth, obs.fctr)
        self.tot_smear = np.sqrt(obs.dt ** 2.0 + (obs.dt * self.downsamp) ** 2.0 +
                                 self.BW_smearing ** 2.0 + self.sub_smearing ** 2.0 +
                                 self.chan_smear ** 2.0)

    def DM_for_smearfact(self, smearfact):
        obs = self.ddplan.obs
        other = np.sqrt(obs.dt ** 2.0 + (obs.dt * self.downsamp) ** 2.0 +
                        self.BW_smearing ** 2.0 + self.sub_smearing ** 2.0)
        return guess_DMstep(smearfact * other, obs.chanwidth, obs.fctr)

    def subband_calls(self):
        """[(subDM, DMs)] of each subband pass: pass k serves the
        DMs_per_prepsub trials starting at loDM + k*dsubDM and is formed at
        subDM = loDM + (k + 0.5)*dsubDM (PRESTO convention; build decision,
        SURVEY.md §3.5)."""
        if not self.numsub:
            return [(None, self.DMs)]
        per = self.DMs_per_prepsub
        return [(self.loDM + (k + 0.5) * self.dsubDM, self.DMs[k * per:(k + 1) * per])
                for k in range(self.numprepsub)]

    def __str__(self):
        if self.numsub:
            return "%9.3f  %9.3f  %6.2f    %4d  %6.2f  %6d  %6d  %6d " % (
                self.loDM, self.hiDM, self.dDM, self.downsamp, self.dsubDM,
                self.numDMs, self.DMs_per_prepsub, self.numprepsub)
        return "%9.3f  %9.3f  %6.2f    %4d  %6d" % (
            self.loDM, self.hiDM, self.dDM, self.downsamp, self.numDMs)


class DDplan(object):
    """A list of DDsteps covering [loDM, hiDM] (DDplan2b.py:202-435)."""

    def __init__(self, loDM, hiDM, obs, numsub=0, resolution=0.0, verbose=False):
        self.loDM = loDM
        self.hiDM = hiDM
        self.obs = obs
        self.numsub = numsub
        self.req_resolution = resolution * 0.001
        self.current_downfact = obs.allow_factors[0]
        self.current_dDM = ALLOW_DMSTEPS[0]
        self.DDsteps = []
        self.calc_min_smearing(verbose)

        while obs.dt * self.get_next_downfact() < self.resolution:
            self.current_downfact = self.get_next_downfact()
        dDM = guess_DMstep(obs.dt * self.current_downfact, 0.5 * obs.BW, obs.fctr)
        while self.get_next_dDM() < dDM:
            self.current_dDM = self.get_next_dDM()
        self.DDsteps.append(DDstep(self, self.current_downfact, self.loDM, self.current_dDM,
                                   numsub=numsub, smearfact=SMEARFACT))
        while self.DDsteps[-1].hiDM < self.hiDM:
            self.current_downfact = self.get_next_downfact()
            eff_dt = obs.dt * self.current_downfact
            while dm_smear(0.5 * self.get_next_dDM(), obs.BW, obs.fctr) < FF * eff_dt:
                self.current_dDM = self.get_next_dDM()
            self.DDsteps.append(DDstep(self, self.current_downfact, self.DDsteps[-1].hiDM,
                                       self.current_dDM, numsub=numsub, smearfact=SMEARFACT))
        wfs = [s.numDMs / float(s.downsamp) for s in self.DDsteps]
        self.work_fracts = np.asarray(wfs) / np.sum(wfs)

    def get_next_dDM(self):
        for d in ALLOW_DMSTEPS:
            if d > self.current_dDM:
                return d
        raise ValueError("No allowable DM steps left!")

    def get_next_downfact(self):
        i = self.obs.allow_factors.index(self.current_downfact)
        if i + 1 < len(self.obs.allow_factors):
            return self.obs.allow_factors[i + 1]
        raise ValueError("No allowable downsample factors left!")

    def calc_min_smearing(self, verbose=False):
        obs = self.obs
        half = 0.5 * ALLOW_DMSTEPS[0]
        self.min_chan_smear = dm_smear(self.loDM + half, obs.chanwidth, obs.fctr)
        self.min_bw_smear = dm_smear(half, obs.BW, obs.fctr)
        self.min_total_smear = np.sqrt(2 * obs.dt ** 2.0 + self.min_chan_smear ** 2.0 +
                                       self.min_bw_smear ** 2.0)
        self.best_resolution = max([self.req_resolution, self.min_chan_smear,
                                    self.min_bw_smear, obs.dt])
        self.resolution = self.best_resolution
        if FF * self.min_chan_smear > obs.dt or self.resolution > obs.dt:
            if not self.resolution > FF * self.min_chan_smear:
                self.resolution = FF * self.min_chan_smear

    @property
    def all_DMs(self):
        return np.concatenate([s.DMs for s in self.DDsteps])

    def __str__(self):
        if self.numsub:
            lines = ["\n  Low DM    High DM     dDM  DownSamp  dsubDM   #DMs  DMs/call  calls  WorkFract"]
        else:
            lines = ["\n  Low DM    High DM     dDM  DownSamp   #DMs  WorkFract"]
        for step, wf in zip(self.DDsteps, self.work_fracts):
            lines.append("%s   %.4g" % (step, wf))
        lines.append("\n")
        return "\n".join(lines)
